"""celestia_da -- MI355X-native celestia-app data-availability hot path.

ODS -> EDS (Leopard RS, GF(2^8)) -> NMT row/column roots -> DAH, on gfx950 HIP
kernels behind the C ABI in include/dagpu.h.  This package is the host-side
mirror of the reference's pkg/da interface (see da.py for the file:line map).
"""
from . import _abi, synth  # noqa: F401
from .da import (  # noqa: F401
    Context,
    DAError,
    DataAvailabilityHeader,
    ErrByzantineData,
    ErrInvalidPushOrder,
    ErrTooFewShards,
    ErrUnrepairableDataSquare,
    ExtendedDataSquare,
    LeoRSCodec,
    default_context,
    extend_batch,
    extend_shares,
    is_power_of_two,
    min_data_availability_header,
    min_shares,
    new_data_availability_header,
    repair,
    nil_dah_hash,
    round_up_power_of_two,
    square_size,
    tail_padding_share,
)

__version__ = "0.1.0"

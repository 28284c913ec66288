// switches.hpp -- the library's environment switches (DAGPU_*).
//
// Every switch selects between two paths that tests/ check against each other
// or against the oracle; none is needed in production.  DESIGN.md §4 "Switches"
// lists each with the A/B log that decided its default.  Superseded kernel
// generations and the switches that lost their A/B are removed from the
// library (round 6), not kept behind a switch.
#pragma once

namespace dagpu {

enum Switch : int {
  SW_PIPELINE_CHUNK,  // squares per host-batch chunk (tests force many chunks)
  SW_PIPE_SLICES,     // RS/NMT pipeline slices of a device batch (1 = off)
  SW_REPAIR_FILL,     // 0: Repair without the fill route (the plain schedule)
  SW_SPLIT_SQUARE,    // 0: the one-part split square through the forest path
  SW_SPLIT_OVERLAP,   // split column encode on a side stream (0 off, 1 high priority, 2 normal)
  SW_DAH_SPLIT,       // 0: the one-stage DAH kernel
  SW_DEC_SLICED,      // 0: the packed GF(2^8) decoder at k = 128
  SW_ENC_SLICED,      // 0: the packed GF(2^8) encoder for k = 16..128
  SW_ENC_SLICED2,     // 0: the four-vector bit-sliced encoder at k = 128
  SW_GF16_WIDE,       // 1: the LDS-slice GF(2^16) kernels at k = 256 / 512 too
  SW_COUNT
};

// The switch's value, nullptr when unset.  Read from the environment on the
// calling thread; a started Repair's worker thread reads the snapshot its
// dagpu_repair_start call took (sw_bind), so no library thread calls getenv
// while the host program may be changing the environment.
const char* sw(Switch s);
// atol of the value; `dflt` when unset
long sw_long(Switch s, long dflt = 0);

struct SwSnapshot {
  bool set[SW_COUNT];
  char v[SW_COUNT][24];
};
void sw_snapshot(SwSnapshot* out);
// this thread reads `snap` from now on (nullptr: the environment again)
void sw_bind(const SwSnapshot* snap);

}  // namespace dagpu

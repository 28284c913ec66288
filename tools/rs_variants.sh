for b in tools/rsb_*; do timeout -k 5 60 $b $(basename $b) || exit 1; done

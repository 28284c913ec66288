# overlap probe: SHA leaf work with a bounded persistent grid (work queue) beside
# RS-shaped work on a second stream, the RS also as a persistent grid (variant 5)
set -o pipefail
out=gpurun_out/overlap_persist.log; : > $out
for p in 2 3 4; do for r in 1 2; do
  timeout -k 5 60 ./tools/overlap_probe 0 5 256 $p 1 $r >> $out 2>&1 || exit 1
done; done
timeout -k 5 60 ./tools/overlap_probe 0 1 256 3 1 >> $out 2>&1 || exit 1
cat $out

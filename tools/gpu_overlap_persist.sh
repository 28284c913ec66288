# overlap probe: SHA leaf-shaped work (flooding grid, or a persistent work-queue grid of P WGs/CU)
# beside RS-shaped work: rs2 (4 waves, 146 VGPRs) and rs6 (8 waves, ~90 VGPRs), flooding or
# persistent (variants 5 / 7, R WGs/CU).  profiles/overlap_queue_r02.log
set -o pipefail
out=gpurun_out/overlap_persist.log; : > $out
timeout -k 5 60 ./tools/overlap_probe 0 1 >> $out 2>&1 || exit 1
timeout -k 5 60 ./tools/overlap_probe 0 6 >> $out 2>&1 || exit 1
for p in 2 3; do
  timeout -k 5 60 ./tools/overlap_probe 0 6 256 $p 1 >> $out 2>&1 || exit 1
  for r in 1 2; do timeout -k 5 60 ./tools/overlap_probe 0 7 256 $p 1 $r >> $out 2>&1 || exit 1; done
done
cat $out

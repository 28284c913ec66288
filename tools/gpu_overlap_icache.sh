# overlap probe: small-code RS work (variant 0) vs ~60 KB straight-line RS code (variant 4) beside
# leaf-shaped SHA work (flooding, or persistent 2/3 WGs per CU): instruction-cache pressure
set -o pipefail
out=gpurun_out/overlap_icache.log; : > $out
for v in 0 4; do for p in 0 2 3; do
  timeout -k 5 60 ./tools/overlap_probe 0 $v 256 $p 1 >> $out 2>&1 || exit 1
done; done
cat $out

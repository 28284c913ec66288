# RS MALL probe + kernel-trace stats of the k=512 and k=128 repair benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rs_mall_probe.py > gpurun_out/rs_mall.log 2>&1; echo "mall rc=$?"; cat gpurun_out/rs_mall.log | tail -9
cd /tmp && export TMPDIR=/tmp
for k in 512 128; do
  b=2; [ $k = 128 ] && b=256
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rep$k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode repair --k $k --batch $b --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/rep$k.log 2>&1
  echo "rep$k rc=$?"; tail -1 $GRAFT_REPO_ROOT/gpurun_out/rep$k.log | cut -c1-220
done

# Build another variant of libdagpu.so for an A/B or a probe run, without
# touching the in-tree build:
#   bash tools/build_variant.sh <name> [<git rev> | -] [extra HIPFLAGS...]
# copies celestia-app_amd + include (the working tree, or `git archive <rev>`)
# to /tmp/dagpu_variant_<name>, builds libdagpu.so there with the extra flags
# (e.g. -DDAGPU_PHASE_PROBE) and installs it as celestia-app_amd/libdagpu_<name>.so
# (GPU runs name it lib:celestia-app_amd/libdagpu_<name>.so; delete it after).
set -e
name=$1; rev=${2:--}; shift 2 || true
root=$(cd "$(dirname "$0")/.." && pwd)
dst=/tmp/dagpu_variant_$name
rm -rf "$dst"; mkdir -p "$dst"
if [ "$rev" = "-" ]; then
  cp -r "$root/celestia-app_amd" "$root/include" "$dst/"
  rm -rf "$dst/celestia-app_amd/build" "$dst/celestia-app_amd/build_test" "$dst/celestia-app_amd/build_asan"
else
  git -C "$root" archive "$rev" celestia-app_amd include | tar -x -C "$dst"
fi
flags="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics $*"
make -s -j8 -C "$dst/celestia-app_amd" libdagpu.so HIPFLAGS="$flags"
cp "$dst/celestia-app_amd/libdagpu.so" "$root/celestia-app_amd/libdagpu_$name.so"
echo "built celestia-app_amd/libdagpu_$name.so ($rev $*)"

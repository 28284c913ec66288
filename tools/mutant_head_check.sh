# Sensitivity check of tests/test_gpu_repair_async.py::test_locator_key_collisions_fall_back_to_own_heads:
# the same collision script against a MUTANT test build whose candidate-head check always
# accepts (err_head_checked_block/_wave return the candidate).  Expected: every Repair wrong.
# Build the mutant first (on the CPU):
#   rm -rf /tmp/mut && mkdir -p /tmp/mut && cp -r celestia-app_amd include /tmp/mut/
#   edit /tmp/mut/celestia-app_amd/csrc/kernels.hpp: "return hv;" unconditionally in both helpers
#   make -C /tmp/mut/celestia-app_amd libdagpu_test.so && cp .../libdagpu_test.so celestia-app_amd/libdagpu_mut.so
# Result round 6: profiles/mutant_head_check_r06.log.
set -o pipefail
python3 - > gpurun_out/r06_mutant.log 2>&1 <<'PY'
import os, re, subprocess, sys
src = open("tests/test_gpu_repair_async.py").read()
script = re.search(r'_KEY_COLLIDE_SCRIPT = r"""(.*?)"""', src, re.S).group(1)
pkg = os.path.abspath("celestia-app_amd")
env = dict(os.environ, DAGPU_LIB=os.path.join(pkg, "libdagpu_mut.so"), DAGPU_TEST_KEY_COLLIDE="1")
r = subprocess.run([sys.executable, "-c", script, pkg], env=env, capture_output=True, text=True, timeout=300)
print("rc", r.returncode)
print(r.stdout)
print(r.stderr[-1500:])
PY
cat gpurun_out/r06_mutant.log | head -20

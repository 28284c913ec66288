# round 4: multi-level forest launches for the upper levels (forest_multi_kernel): tests, then split A/B by threshold
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_trees.py tests/test_gpu_split.py tests/test_gpu_proof.py tests/test_gpu_inclusion.py tests/test_gpu_c_client.py" --rounds 2 split512 m64= m32=DAGPU_FOREST_MULTI=32 m128=DAGPU_FOREST_MULTI=128 single=DAGPU_FOREST_MULTI=0

# native URDF load on the GPU + physics / edge suites (developer session)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3t; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_physics.py tests/test_gpu_edge.py -m gpu -v --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" $OUT/tests.log | tail -20

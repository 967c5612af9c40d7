set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/dgin
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "dgrad_refl_in_fused or dgrad_reflect_border" > gpurun_out/dgin/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/dgin/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/dgin/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_models.py -k "full_size_train_step" > gpurun_out/dgin/pytest2.log 2>&1; rc=$?; tail -3 gpurun_out/dgin/pytest2.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/dgin/pytest2.log | head -20; exit $rc; }
ARMS="default VST_DGRAD_IN=0" TAG=dgin bash tools/ab_step.sh

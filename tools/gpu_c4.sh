set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "c4_direct or four_channel or dgrad_as_fprop" > gpurun_out/c4/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/c4/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/c4/pytest.log | head -20; exit $rc; }
KB_B=8 timeout -k 10 200 python -u tools/kbench_time.py > gpurun_out/c4/kb.json 2>gpurun_out/c4/kb.err; tail -2 gpurun_out/c4/kb.json
VST_C4_DIRECT=0 KB_B=8 timeout -k 10 200 python -u tools/kbench_time.py > gpurun_out/c4/kb0.json 2>gpurun_out/c4/kb0.err; tail -2 gpurun_out/c4/kb0.json

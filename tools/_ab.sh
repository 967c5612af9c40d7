set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab5; mkdir -p $O
V=gan-based-video-style-transfer_amd/_build/variants
for v in st1 st1s0 st1r1 s0 st1r1s0 st1 st1s0 st1r1 s0 st1r1s0; do
  if [ $v = default ]; then L=""; else L=$V/lib_$v.so; fi
  VST_LIB_VARIANT=$L timeout -k 10 120 python tools/kbench_time.py >> $O/kb.log 2>&1 || { echo kb fail; tail $O/kb.log; exit 1; }
done
grep -v amdgpu.ids $O/kb.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['lib'][-12:], ' '.join('%s=%s' % (k[:-3], v) for k, v in d.items() if k.endswith('_us')))"

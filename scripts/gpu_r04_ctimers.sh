# round 4: the one-frame parse's phase cycles (tuning build, ZSEEK_CHUNK_TIMERS)
# at lead-ins of 0 / 64 / 128 bytes, then the GPU suite and the latency probe
# (product build, default lead-in, per-wave match passes in the execute)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for L in 0 64 128; do
ZSEEK_ONE_LEAD=$L ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 > gpurun_out/ctimers$L.log 2>&1 || { tail -5 gpurun_out/ctimers$L.log; exit 1; }
echo "lead $L"; grep "chunk one-route" gpurun_out/ctimers$L.log | tail -1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ct_suite.log 2>&1 || { tail -30 gpurun_out/ct_suite.log; exit 1; }
tail -1 gpurun_out/ct_suite.log
timeout -k 10 300 python scripts/latency_probe.py 300 2>&1 | grep p50
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-verify > gpurun_out/ct_bench.json 2> gpurun_out/ct_bench.err || { tail -5 gpurun_out/ct_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/ct_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['latency_4k_us'])"

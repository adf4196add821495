# GPU LZ4 compression A/B: parity tests, then one bench line per probe batch size
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lz4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lz4_compress.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for P in ${1:-8 16 32}; do
  ZSEEK_LZ4C_PROBE=$P timeout -k 10 300 python bench.py --codec lz4c --steps 5 --warmup 2 --no-cpu-baseline --no-verify > $O/ab$P.json 2> $O/ab$P.log || { tail -20 $O/ab$P.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab$P.json'));print('probe $P', d['value'], d['ms_per_step'])"
done

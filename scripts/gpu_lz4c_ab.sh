# GPU LZ4 compression A/B: parity tests (default variant and each variant's
# kernel through the oracle tests), then one bench line per variant
# "PROBES:VAL" (ZSEEK_LZ4C_PROBE / ZSEEK_LZ4C_VAL, tuning only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lz4c
mkdir -p $O
for V in ${1:-8:0 8:1}; do
  P=${V%%:*}; L=${V##*:}
  ZSEEK_LZ4C_PROBE=$P ZSEEK_LZ4C_VAL=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lz4_compress.py > $O/tests_${P}_${L}.log 2>&1 || { tail -30 $O/tests_${P}_${L}.log; exit 1; }
  echo "variant $V: $(tail -1 $O/tests_${P}_${L}.log)"
  ZSEEK_LZ4C_PROBE=$P ZSEEK_LZ4C_VAL=$L timeout -k 10 300 python bench.py --codec lz4c --steps 5 --warmup 2 --no-cpu-baseline --no-verify --profile > $O/ab.json 2> $O/ab.log || { tail -20 $O/ab.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab.json'));print('variant $V', d['value'], d['ms_per_step'])"
done

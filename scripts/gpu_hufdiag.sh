# zstd Huffman kernel elimination diagnostics (ZSEEK_ZSTD_HUF_DIAG: 1 = no
# literal stores, 3 = also no chunk loads, 7 = also no table lookups): the
# kernel's time from a rocprofv3 kernel trace of one bench launch each (the
# decoded output is wrong under a diagnostic, so the bench stops after it).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/hufdiag
mkdir -p $O
for dg in 0 1 3 7; do
  ZSEEK_ZSTD_HUF_DIAG=$dg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$dg -- python bench.py --codec zstd --profile --steps 1 --warmup 1 --no-e2e > $O/d$dg.log 2>&1
  rc=$?
  if [ $rc -ge 124 ]; then echo "diag $dg: rc $rc"; exit 1; fi
  python - "$O/d$dg" "$dg" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/*/*_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "zstd_huf" in r["Name"] or "zstd_seq" in r["Name"]:
            print("diag", sys.argv[2], r["Name"][30:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), round(float(r["MinNs"]) / 1e6, 3))
PY
done

# FETCH_SIZE / WRITE_SIZE calibration on the execute's access pattern
# (scripts/fetch_calib.py): one workload run, one --pmc pass per counter.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fcalib}
mkdir -p $O
timeout -k 10 300 python scripts/fetch_calib.py --meta $O/meta.json > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
cat $O/run.log
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -- python scripts/fetch_calib.py > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -- python scripts/fetch_calib.py > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
python scripts/fetch_calib.py --summarize $O > $O/calib.json && cat $O/calib.json

# one probe mode per call (a crash ends the call): bash gpu_hang_probe.sh MODE [ITERS]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/probe
mkdir -p $O
M=${1:-both}
timeout -k 10 150 python -u scripts/hang_probe.py $M ${2:-60} > $O/$M${3:-}.log 2>&1
rc=$?
grep -c "^iter" $O/$M${3:-}.log
tail -4 $O/$M${3:-}.log
exit $rc

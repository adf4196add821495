# round 4: production execute (3,584-byte stage) against the 4,096 stage on a
# fresh tuning build; the GPU suite and the churn probe with streams / events
# destroyed by default (ZSEEK_HIP_POOL unset).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04combo3
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 0,321 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep -v amdgpu.ids $O/kb.log | grep "median\|MISMATCH\|bit-exact"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python -u scripts/hang_probe.py both 250 > $O/probe.log 2>&1
rc=$?
tail -3 $O/probe.log
echo "probe rc=$rc"
[ $rc -eq 0 ] || exit 0

# execute VALU per wave by section on the new build (variant 12 = plan+parse
# only, 20 = execute alone; 0x108/0x104/0x122 drop round 0 / rounds / flush;
# 0x301/0x302/0x304/0x307 parts of the rounds); 0x110 = section cycles
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -- python scripts/kbench.py --variants 12,20,264,260,290,769,770,772,775 --rounds 1 --reps 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/r04combo3/p1/*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'seq_exec' not in r['Kernel_Name']:
            continue
        k = (r['Kernel_Name'][:90], int(r['Dispatch_Id']))
        rows[k][r['Counter_Name']] += float(r['Counter_Value'])
for k in sorted(rows, key=lambda x: x[1]):
    c = rows[k]; w = c['SQ_WAVES']
    print(k[1], k[0][40:90], 'per-wave VALU %.0f SALU %.0f LDS %.0f BR %.0f cyc %.0f active %.0f wait %.0f' % (
        c['SQ_INSTS_VALU']/w, c['SQ_INSTS_SALU']/w, c['SQ_INSTS_LDS']/w, c['SQ_INSTS_BRANCH']/w,
        c['SQ_WAVE_CYCLES']/w, c['SQ_ACTIVE_INST_ANY']/w, c['SQ_WAIT_ANY']/w))
PY
timeout -k 10 300 python scripts/kbench.py --variants 20,800,832,864,769,770,264,260,290,272 --rounds 3 > $O/kb2.log 2>&1 || { tail -20 $O/kb2.log; exit 1; }
grep "median\|exec sections\|per batch\|MISMATCH\|bit-exact" $O/kb2.log | sort | uniq | head -20
exit 0

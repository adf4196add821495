# execute-kernel VALU / SALU / LDS instructions per wave by section: the
# tuning build's elimination variants (execute alone over the items of a
# prior plan + lean parse, variant 12): 20 = whole, 0x108 = no round 0,
# 0x104 = no dependency rounds, 0x122 = no flush.  One PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04xvalu
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -- python scripts/kbench.py --variants 12,20,264,260,290,769,770,772,775 --rounds 1 --reps 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/r04xvalu/p1/*/*_counter_collection.csv'):
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
timeout -k 10 300 python scripts/kbench.py --variants 12,20,769,770,772,775,264,260 --rounds 3 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep median $O/kb.log

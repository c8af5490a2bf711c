set -o pipefail
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/rtpmc
mkdir -p $base
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY TA_TA_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $base/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $base/p3 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/p3.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections
for p in ('p2', 'p3'):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f'/root/repo/gpurun_out/rtpmc/{p}/run_counter_collection.csv')):
        k = r['Kernel_Name']
        if not (('rowtile' in k and 'true' in k) or 'dw_kernel' in k): continue
        k = ('actorT' if 'actor' in k else 'criticT' if 'critic' in k else 'dw')
        acc[(k, r['Counter_Name'])] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
    for (k, c), v in sorted(acc.items()): print(p, k, c, round(v / n[(k, c)]))
PY

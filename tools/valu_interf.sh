# Does the memory traffic make the stream kernel's VALU instructions cost more cycles?
# PMC of the C2 seal/open kernels with and without the memory waves' traffic (ENET_STREAM_DBG=1).
export TMPDIR=/tmp
O=gpurun_out/vi; mkdir -p $O
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for D in 0 1; do
  ENET_STREAM_DBG=$D timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/d$D -o p -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > /dev/null 2>&1 || exit 1
done
C2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
for D in 0 1; do
  ENET_STREAM_DBG=$D timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d $O/e$D -o p -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv,glob,collections
for tag in ('d0','d1','e0','e1'):
    d=collections.defaultdict(list); dur=[]
    for f in glob.glob(f'gpurun_out/vi/{tag}/**/p_counter_collection.csv',recursive=True):
        for r in csv.DictReader(open(f)):
            if 'stream_kernel<1, 1' in r['Kernel_Name']:
                d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(tag, {k: round(sum(v)/len(v)) for k,v in sorted(d.items())})
PY

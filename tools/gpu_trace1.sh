set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
rm -rf gpurun_out/pt
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/pt -o run --output-format csv -- python3 tools/run_ops.py --op both --iters 3 > gpurun_out/pt.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
t = glob.glob('gpurun_out/pt/**/run_kernel_trace.csv', recursive=True)[0]
for r in csv.DictReader(open(t)):
    if 'k200' in r['Kernel_Name']:
        print(r['Kernel_Name'][:40], 'grid', r.get('Grid_Size'), r.get('Grid_Size_X'), 'wg', r.get('Workgroup_Size'), r.get('Workgroup_Size_X'), 'lds', r.get('LDS_Block_Size'), r.get('Lds_Size'), 'vgpr', r.get('VGPR_Count'), 'dur', int(r['End_Timestamp'])-int(r['Start_Timestamp']))
        break
print(list(r.keys()))
PY
tools/gpu_traffic_ab.sh main

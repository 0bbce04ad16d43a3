set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/jt -o jt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --large-trees 0 --predict-trees 0 --hessian 0 --c3-evals 0 --example-mp 0 --c4-trees 0 --c5-trees 0 --example-parity 0 > gpurun_out/jt.json 2> gpurun_out/jt.err || { tail -5 gpurun_out/jt.err; exit 1; }
python3 - <<'P'
import csv, glob
f = glob.glob('gpurun_out/jt/**/*kernel_trace.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'joint' in r['Kernel_Name']:
        print(r['Kernel_Name'][:40], r['Grid_Size'] if 'Grid_Size' in r else r.get('Grid_Size_X'), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, 'us')
P

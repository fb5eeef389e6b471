set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/c4w; cd /tmp && export TMPDIR=/tmp
for a in "" "--no-records" "--no-svc-dur"; do
n=$(echo "x$a" | tr -d ' -'); 
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/c4w/$n -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --no-cpu $a > $R/gpurun_out/c4w/$n.log 2>&1 || exit 14
python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/c4w/$n/**/*counter_collection.csv',recursive=True)[0]
v=[float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'isim_tree' in r['Kernel_Name'] and r['Counter_Name']=='WRITE_SIZE']
print('$a', 'WRITE_SIZE KB per launch', sum(v)/len(v))"
done

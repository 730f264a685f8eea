# rocprofv3 kernel stats of the detector API bench (worker process included), top kernels by total time
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pdet
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pdet -o run -- python -u bench/api_bench.py --model detector --steps 20 --warmup 3 > gpurun_out/pdet/log 2>&1 || { tail -5 gpurun_out/pdet/log; exit 1; }
f=$(find gpurun_out/pdet -name "*kernel_stats.csv" | head -1)
python -c "
import csv
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
print('total ms', round(tot/1e6,1))
for r in rows[:30]: print(round(float(r['TotalDurationNs'])/1e3,1), r['Calls'], round(float(r['TotalDurationNs'])/tot*100,1), r['Name'][:110])
"

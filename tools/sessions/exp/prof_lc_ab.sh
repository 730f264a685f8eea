# per-kernel time of the land-cover forward: default kernel library vs an experiment library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for tag in new old; do
  lib=""; [ $tag = old ] && lib="$1"
  AI4E_KERNEL_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/prof_$tag -o run -- python -u bench/landcover_bench.py --steps 4 --warmup 1 > gpurun_out/exp/prof_$tag.log 2>&1 || { tail -5 gpurun_out/exp/prof_$tag.log; exit 1; }
done
for tag in new old; do echo "== $tag"; f=$(find gpurun_out/exp/prof_$tag -name "*kernel_stats.csv" | head -1); python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:14]: print(round(float(r['TotalDurationNs'])/1e3,1), r['Calls'], r['Name'][:90])
"; done

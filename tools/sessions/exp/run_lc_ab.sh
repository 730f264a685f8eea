# land-cover forward bench with the default kernel library vs an experiment library, alternating
set -o pipefail
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for r in 1 2 3; do
for lib in "" "$1"; do
  AI4E_KERNEL_LIB=$lib timeout -k 10 200 python -u bench/landcover_bench.py --steps 8 > gpurun_out/exp/lc.log 2>&1 || { tail -5 gpurun_out/exp/lc.log; exit 1; }
  echo "lib=${lib:-default} $(grep '^{' gpurun_out/exp/lc.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_mosaic'])")"
done
done

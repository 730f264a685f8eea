# chain_tune timings (B=250) with the default kernel library and experiment libraries (tools/sessions/exp/*.so)
set -o pipefail
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for lib in "" "$@"; do
  echo "== lib=${lib:-default}"
  AI4E_KERNEL_LIB=$lib B=250 timeout -k 10 200 python -u bench/chain_tune.py > gpurun_out/exp/chain.log 2>&1 || { tail -5 gpurun_out/exp/chain.log; exit 1; }
  grep '^{' gpurun_out/exp/chain.log
done

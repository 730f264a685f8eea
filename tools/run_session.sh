#!/bin/bash
# Same-box A/B session: each "label|env assignments|seconds|command" line of $AB_FILE runs under its own time limit,
# writes gpurun_out/ab_<label>.log, and the session stops at the first failure (no retries on the GPU).
#   AB_FILE=tools/sessions/ab_r4m.txt bash tools/run_session.sh   (round files: tools/sessions/ab_r*.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
while IFS='|' read -r label envs secs cmd; do
  [ -z "$label" ] && continue
  case "$label" in \#*) continue ;; esac
  echo "=== $label: $envs $cmd"
  env $envs timeout -k 10 "$secs" $cmd < /dev/null > "gpurun_out/ab_${label}.log" 2>&1
  rc=$?
  grep '^{' "gpurun_out/ab_${label}.log" | tail -1 | cut -c1-400
  echo "=== $label rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/ab_${label}.log"; echo "STOP after $label"; exit $rc; fi
done < "${AB_FILE:?set AB_FILE to a session file (tools/sessions/ab_r*.txt)}"
echo "=== done"

#!/bin/bash
# Build an experiment variant of the kernel library: all csrc/kernels sources, with the listed
# replacements from tools/sessions/exp/ (timing experiments only; loaded through AI4E_KERNEL_LIB).
#   tools/sessions/exp/build_exp.sh <out.so> <kernel-name=replacement.hip>...
set -e
cd "$(dirname "$0")/../.."
out=$1; shift
objs=()
mkdir -p tools/sessions/exp/obj
for src in csrc/kernels/*.hip; do
  name=$(basename "$src" .hip)
  for r in "$@"; do [ "${r%%=*}" = "$name" ] && src="tools/sessions/exp/${r#*=}"; done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 \
    -Wno-unused-result -Icsrc/kernels -c "$src" -o "tools/sessions/exp/obj/$name.o" &
  objs+=("tools/sessions/exp/obj/$name.o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o "$out"

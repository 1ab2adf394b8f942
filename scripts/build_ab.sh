#!/bin/bash
# Build an A/B variant of the kernel library with some source files taken from a git revision:
#   scripts/build_ab.sh <rev> <name> <csrc/kernels/file.hip> [more files...]
# Headers (*.h) listed are taken from <rev> too and shadow the tree's for the listed sources.
# -> databricks_distributed_deep_learning_amd/_native/ab/libddl_<name>.so (load with DDL_NATIVE_LIB=...)
set -euo pipefail
rev=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/databricks_distributed_deep_learning_amd/_native/ab
tmp=$(mktemp -d)
mkdir -p "$out"
python "$root/csrc/build.py" >/dev/null
declare -A swap
mkdir -p "$tmp/include"
for src in "$@"; do
  case $src in *.h) git -C "$root" show "$rev:$src" > "$tmp/include/$(basename "$src")";; esac
done
for src in "$@"; do
  case $src in *.h) continue;; esac
  b=$(basename "$src")
  git -C "$root" show "$rev:$src" > "$tmp/$b"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$tmp/include" -I "$root/csrc/include" -Wno-unused-result \
      -ffp-contract=fast -munsafe-fp-atomics -c "$tmp/$b" -o "$tmp/$b.o"
  swap[$b.o]=$tmp/$b.o
done
objs=()
for o in "$root"/build/native/*.o; do
  b=$(basename "$o")
  objs+=("${swap[$b]:-$o}")
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o "$out/libddl_$name.so" \
    -L/opt/rocm/lib -Wl,--no-as-needed -lamdhip64 -ldl
rm -rf "$tmp"
echo "$out/libddl_$name.so"

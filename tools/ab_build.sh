#!/bin/bash
# Build variants of the assembly interpreter (generator knobs passed as env assignments) into
# ab/<name>.so for A/B benches on one GPU box (bench.py picks one with EBPF_LIB=...).
#   tools/ab_build.sh name "EBPF_ASM_RETK=8 EBPF_ASM_NT=3" [name2 "env2" ...]
# The default build is restored at the end.
set -e
cd "$(dirname "$0")/.."
mkdir -p ab
while [ $# -ge 2 ]; do
  touch generic-ebpf_amd/csrc/asm/gen_interp.py
  env $2 make -s -j8 -C generic-ebpf_amd > /dev/null
  cp generic-ebpf_amd/lib/libebpf.so ab/$1.so
  echo "built ab/$1.so ($2)"
  shift 2
done
touch generic-ebpf_amd/csrc/asm/gen_interp.py
make -s -j8 -C generic-ebpf_amd > /dev/null

#!/bin/bash
# Ablation: same sweep against alternative builds of libmrt.so in abl/<name>/.
for v in "" $(ls abl); do
  echo "== variant ${v:-current}"
  if [ -n "$v" ]; then export MRT_LIB_DIR=$PWD/abl/$v; else unset MRT_LIB_DIR; fi
  timeout -k 10 200 python tools/sweep.py --workloads "$1" --configs "$2" --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done

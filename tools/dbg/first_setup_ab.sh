#!/bin/bash
# first sparse setup of a fresh process (learn_twice run 0) and the second, base library vs the in-tree one, alternating
set -e
o=gpurun_out/fs; mkdir -p $o
for rep in 1 2 3; do
  for v in base cur; do
    lib=""; [ $v = base ] && lib=$PWD/variants/base/libplssvm_mi355x.so
    for c in csr_rbf_1m fp22_rbf_2m; do
      PLSSVM_MI_LIB=$lib timeout -k 10 300 python -u tools/dbg/learn_twice.py $c 2>/dev/null | grep learn_s | sed "s/^/$v /" >> $o/res.txt
    done
  done
done
cat $o/res.txt

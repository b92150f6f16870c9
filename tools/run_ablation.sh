#!/bin/bash
for v in BASE STUB_TAN STUB_ATAN STUB_HYP STUB_EXP; do
  echo "== $v" >> gpurun_out/ablation.log
  timeout -k 10 120 ./tools/gv_$v 1024 512 4000 2>&1 | head -1 >> gpurun_out/ablation.log || exit 1
done

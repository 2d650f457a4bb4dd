#!/bin/bash
# A/B the x6 convolutions of several variant builds on the step's shapes:
#   tools/ab_conv.sh MODES name1 name2 ...
set -o pipefail
modes=$1; shift
for v in "$@"; do
  echo "== $v"
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 5 300 python tools/conv_x6_bench.py $modes || exit 1
done

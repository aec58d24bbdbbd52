#!/bin/bash
# Same-box A/B of two library builds: runs `python <script> <args>` alternately with ADP_LIB_PATH = A and B
# (R rounds, ABAB...), each output line prefixed with the arm. GPU box, repo root.
# usage: bash tools/ab_libs.sh <libA.so> <libB.so> <rounds> <script.py> [args...]
set -uo pipefail
A=$1; B=$2; R=$3; shift 3
for r in $(seq 1 "$R"); do
  for arm in A B; do
    lib=$A; [ $arm = B ] && lib=$B
    ADP_LIB_PATH=$lib timeout -k 10 300 python "$@" 2>/dev/null | sed "s/^/$arm r$r /" || { echo "$arm r$r failed"; exit 1; }
  done
done

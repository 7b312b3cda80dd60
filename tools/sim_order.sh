#!/bin/bash
# Rank shares of a W-GPU job timed in a given order (thermal / ordering check for tools/sim_shares.sh).
# usage: tools/sim_order.sh <config> <W> <rank> [rank ...]
config=$1; W=$2; shift 2
for r in "$@"; do
  timeout -k 10 120 python bench.py --config "$config" --sim-rank "$r/$W" --steps 20 --warmup 1 --no-cpu 2>/dev/null || exit $?
done

#!/bin/bash
# A/B of library builds, alternating, N rounds: tools/ab.sh OUT.jsonl ROUNDS name1 name2 ...
set -o pipefail
OUT=$1; R=$2; shift 2
for i in $(seq $R); do tools/variant_bench.sh $OUT "$@" || exit 1; done

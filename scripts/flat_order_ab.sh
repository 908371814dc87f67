#!/usr/bin/env bash
# k_flat2 group order A/B on the mixed batch (GPU box): LVLIP_FLAT_GROUPS is
# read once per process, so every variant runs as its own bench process,
# interleaved over ROUNDS rounds.  Prints one "variant value" line per run.
#   ROUNDS=3 UNROLLS="8 4" bash scripts/flat_order_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=${ROUNDS:-3}
UNROLLS=${UNROLLS:-8}
ORDERS=${ORDERS:-quarters block}
for r in $(seq "$ROUNDS"); do
    for u in $UNROLLS; do
        for o in $ORDERS; do
            v=$(LVLIP_FLAT_GROUPS=$o timeout -k 10 120 python3 bench.py --workload mixed --kernel flat \
                --unroll "$u" --no-cpu-baseline 2>/dev/null |
                python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["value"])')
            rc=$?
            if [ $rc -ne 0 ]; then echo "run failed rc=$rc ($o u$u)"; exit $rc; fi
            echo "round $r u$u $o $v"
        done
    done
done

#!/bin/bash
# Headline A/B: network rounds signalled by a torch event (UTTT_ROUND_EVENTS=1) or by the ring tag (default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-events}
mkdir -p $OUT
for i in 1 2 3; do
  for e in 1 0; do
    UTTT_ROUND_EVENTS=$e timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 \
      --warmup 4 > $OUT/head_e${e}_$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('events', sys.argv[2], d['value'])" $OUT/head_e${e}_$i.log $e
  done
done

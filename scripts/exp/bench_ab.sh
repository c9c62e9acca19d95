#!/bin/bash
# Interleaved single-shot bench.py windows through loopback in the peers'
# schedule: auto opening choice vs forced serial opening (--no-frame-overlap).
#   bash scripts/exp/bench_ab.sh TILE REPS OUT
tile=$1 reps=$2 out=$3
mkdir -p "$(dirname "$out")"
: > "$out"
for i in $(seq "$reps"); do
  for mode in auto serial; do
    extra=""; [ "$mode" = serial ] && extra="--no-frame-overlap"
    MXS_PEER_SCHEDULE=1 timeout -k 10 200 python bench.py --global "$tile" --loopback --steps 20 --warmup 5 --no-extras $extra \
      2>/dev/null | grep "^{" | python -c "
import json, sys
d = json.loads(sys.stdin.read()); e = d['extras']
print(json.dumps({'mode': '$mode', 'tile': e['tile'], 'window_ms': round(d['ms_per_step'] * 20, 4), 'halo_last': e['halo_last'],
                  'outer': e.get('schedule_choice', {}).get('opening_outer_wgs')}))" >> "$out" || exit 1
  done
done
python - "$out" <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
for m in ("auto", "serial"):
    v = sorted(r["window_ms"] for r in rs if r["mode"] == m)
    print(m, "n", len(v), "median", v[len(v) // 2], "min", v[0], "max", v[-1], "halo_last", sum(r["halo_last"] for r in rs if r["mode"] == m))
PY

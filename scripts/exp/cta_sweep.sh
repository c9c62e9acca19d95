# The interior-first opening's exchange with the halo communicator's CTA cap:
# interleaved single-shot bench-flow windows (8-GPU tile, loopback, peers'
# schedule) for caps 0 (RCCL default), 8, 16, 32 -> gpurun_out/r04_cta/cta.jsonl
set -uo pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_cta; mkdir -p $O; : > $O/cta.jsonl
reps=${1:-4}
for i in $(seq $reps); do
  for c in 0 8 16 32; do
    timeout -k 10 200 python bench.py --global 16384x8192 --loopback --rehearse-peers --steps 20 --warmup 5 \
      --no-extras --halo-max-ctas $c > $O/last.txt 2>&1 || { echo "cta $c failed"; tail -20 $O/last.txt; exit 1; }
    python - $O/last.txt $c >> $O/cta.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); e = d["extras"]
print(json.dumps({"cap": int(sys.argv[2]), "window_ms": round(d["ms_per_step"] * 20, 4), "opening": e["opening"],
                  "ratio": e["schedule_choice"].get("ratio"), "phases": e["window_phases"]["phases_us"],
                  "span": e["window_phases"]["gpu_span_us"]}))
PY
  done
done
python - $O/cta.jsonl <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
for c in (0, 8, 16, 32):
    v = sorted(r["window_ms"] for r in rs if r["cap"] == c)
    rat = sorted(r["ratio"] for r in rs if r["cap"] == c)
    print(c, "median", v[len(v) // 2], "min", v[0], "ratios", rat)
PY

set -e
for a in "" "--greedy-flags 1 --topk 256"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --greedy-steps 2 $a > gpurun_out/cfg.json 2> gpurun_out/cfg.err
  python3 - "$a" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/cfg.json").read().strip().splitlines()[-1])
print(repr(sys.argv[1]), "1M:", round(d["greedy"]["gang_placements_per_s"]), {k: (round(v["gang_placements_per_s"]), round(v["ms_per_batch"], 1), v["windows_per_batch"], v["rescans_per_batch"]) for k, v in d["configs"].items()})
PY
done

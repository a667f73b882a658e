"""Walk kernel A/B across library builds (PE_LIBRARY), one box, interleaved: the bench's greedy batch
(cfg3 mix, 1M nodes) -- batch time, host / wait, walk kernel time per launch (hipEvents pass).
    python tools/walk_ab.py lib1.so lib2.so ...   ("" = the in-tree library)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for rep in range(2):
    for lib in sys.argv[1:]:
        env = dict(os.environ)
        if lib:
            env["PE_LIBRARY"] = os.path.abspath(lib)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-configs",
                            "--steps", "1", "--warmup", "1", "--greedy-steps", "3"], env=env, capture_output=True,
                           text=True, timeout=300, cwd=ROOT)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode or not line:
            print(lib, "FAILED", p.stderr[-2000:], flush=True)
            sys.exit(1)
        g = json.loads(line[0])["greedy"]
        r = g.get("roofline", {})
        w = r.get("warm", {}).get("events_walk_ms_per_batch", 0)
        c = r.get("cold", {}).get("events_walk_ms_per_batch", 0)
        n = max(1, g["windows_per_batch"])
        print(f'{os.path.basename(lib) or "libplacement.so":<16} {g["ms_per_batch"]:6.2f} ms/batch host '
              f'{g["host_resolve_ms_per_batch"]:.2f} wait {g["device_wait_ms_per_batch"]:.2f} walk warm '
              f'{w * 1e3 / n:.1f} us/launch cold {c * 1e3 / n:.1f} us/launch rounds/grp {r.get("rounds_per_group", 0):.2f} '
              f'jobs_placed {g["jobs_placed"]}', flush=True)

#!/usr/bin/env python3
"""pe_pg_min_resources calls for the aggregation profile pass (profiles/run_profile.sh): the bench's
1M-job v1 batch, 5 calls after 2 warm-ups, so rocprofv3's pg_agg_seg_kernel average is the 1M-job
launch the bench's aggregation roofline times with hipEvents."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]
from placement import Engine, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
eng = Engine(0)
agg = synth.make_pg_batch(n, synth.SEED["cfg3"])
for _ in range(7):
    eng.pg_min_resources(1, *agg)
eng.close()
print(f"aggregation calls done ({n} jobs)")

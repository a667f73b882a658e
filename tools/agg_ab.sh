set -e
for i in 1 2 3; do for v in vold vnew; do
  PE_LIBRARY=$PWD/build_variants/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --steps 2 --warmup 1 > gpurun_out/aab.json 2> gpurun_out/aab.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/aab.json').read().strip().splitlines()[-1]); a=d['aggregation']; e=d['fit_end_to_end']
print('$v', 'agg %.3f ms %.3g jobs/s' % (a['ms_per_call'], a['jobs_per_s']), 'e2e %.3f upload %.3f' % (e['ms_per_batch'], e['upload_ms']), flush=True)"
done; done

for tk in 32 64 128 256; do for wg in 32 64 128; do
  line=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --steps 1 --warmup 0 --greedy-steps 2 --topk $tk --window-groups $wg)
  python3 -c "
import json,sys
d=json.loads(sys.argv[1]); g=d['greedy']
print('topk=$tk wg=$wg', round(g['ms_per_batch'],1), 'ms windows', g['windows_per_batch'], 'rescans', g['rescans_per_batch'], 'wait', round(g['device_wait_ms_per_batch'],1), 'host', round(g['host_resolve_ms_per_batch'],1))" "$line"
done; done

set -e
export TMPDIR=/tmp
for f in 0 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --greedy-steps 3 --greedy-flags $f > gpurun_out/gb_$f.json 2> gpurun_out/gb_$f.err
done
rm -rf gpurun_out/walkprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/walkprof -o t --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --greedy-steps 2 > gpurun_out/walkprof.json 2> gpurun_out/walkprof.err

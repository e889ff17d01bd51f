cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/st
for np in ${NPS:-1048576 1228800 524288 1310720}; do
  timeout -k 10 200 python -u bench.py --config 4 --order round_robin --packets $np --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/st/$np.json 2>gpurun_out/st/err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/st/$np.json').read().strip().split(chr(10))[-1]); print($np, $np//4096, d['value'], d['kernels_ms'])"
done

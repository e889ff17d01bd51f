cd $GRAFT_REPO_ROOT
for sc in "2 8" "4 16" "4 32" "8 32" "3 12"; do set -- $sc
  timeout -k 10 200 python -u bench.py --packets 1048576 --steps 5 --warmup 2 --cpu-seconds 0 --e2e --e2e-streams $1 --e2e-chunks $2 > gpurun_out/e2e_$1_$2.json 2>gpurun_out/e2e.err || { tail gpurun_out/e2e.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/e2e_$1_$2.json')); print('$1 $2', d['e2e'])"
done

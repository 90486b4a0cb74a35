set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/exp_parity.log 2>&1 || { tail -20 gpurun_out/exp_parity.log; exit 1; }
tail -2 gpurun_out/exp_parity.log
for i in 1 2; do timeout -k 10 200 python bench.py --no-train --no-c5 --no-cpu-baseline --steps 2000 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels_ms'])"; done
timeout -k 10 200 python bench.py --no-train --no-c5 --no-cpu-baseline --num-envs 32768 --level 9 --steps 300 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels_ms'])"

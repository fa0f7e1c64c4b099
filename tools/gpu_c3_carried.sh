cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_slide_carried_gpu.py tests/test_gpu_parity.py tests/test_bench_shapes_gpu.py > gpurun_out/r05_carried_tests.log 2>&1 || { tail -40 gpurun_out/r05_carried_tests.log; exit 1; }
tail -1 gpurun_out/r05_carried_tests.log
for rep in 1 2; do for v in 0 1; do
  timeout -k 10 300 python -u bench.py --config c3 --warmup 2 --option slide_carried=$v > gpurun_out/r05_c3_carried${v}_$rep.json 2> gpurun_out/r05_c3_carried${v}_$rep.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_c3_carried${v}_$rep.json').read().strip().splitlines()[-1]); print('carried=$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'fire %.3f' % d['roofline_fire']['ms_per_step'])"
done; done

#!/bin/bash
# r05: combine3 launch geometry A/B (spill-free builds): parity with forced window passes, then C2 / C3 / C5 benches,
# for each library given (default: the three r05 variants). Each GPU step has its own time limit; the first failure ends the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp flink_amd/libflink_amd.so flink_amd/libflink_amd_base.so
for L in ${LIBS:-base t512 t1024s}; do
  cp flink_amd/libflink_amd_$L.so flink_amd/libflink_amd.so || exit 1
  echo "== $L parity (window passes forced)"
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "random_streams" --force-option window_passes=1 > gpurun_out/r05_ab_${L}_parity.log 2>&1 || { tail -20 gpurun_out/r05_ab_${L}_parity.log; exit 1; }
  tail -1 gpurun_out/r05_ab_${L}_parity.log
  timeout -k 10 200 python -u tests/forced_modes_check.py > gpurun_out/r05_ab_${L}_forced.log 2>&1 || { tail -20 gpurun_out/r05_ab_${L}_forced.log; exit 1; }
  tail -1 gpurun_out/r05_ab_${L}_forced.log
  for c in c2 c3 c5; do
    w=1; [ $c = c3 ] && w=2
    timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup $w --no-cpu-baseline --no-pcie --no-wire \
      > gpurun_out/r05_ab_${L}_$c.json 2> gpurun_out/r05_ab_${L}_$c.log || { tail -5 gpurun_out/r05_ab_${L}_$c.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05_ab_${L}_$c.json')); print('$L $c', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k: round(v/10,3) for k,v in d['ingest_split_ms'].items()}, 'fire/step %.3f'%(d['fire']['ms']/10), 'replay', d['roofline']['replay_records'])"
  done
done

#!/bin/bash
# A/B of two builds of the engine on one box: flink_amd/libflink_amd.so (A, the working tree) against
# flink_amd/libflink_amd_base.so (B, e.g. built from the previous commit with `make OUT=../libflink_amd_base.so`),
# alternating REPS times on the bench config CFG (default c2). The box's copy of the library file is swapped between
# runs; the tree here is untouched. TAG names the outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ablib}; REPS=${REPS:-3}; CFG=${CFG:-c2}; ARGS=${ARGS:-}
L=flink_amd/libflink_amd.so
cp $L /tmp/fwa_a.so && cp flink_amd/libflink_amd_base.so /tmp/fwa_b.so || exit 1
for rep in $(seq $REPS); do for v in a b; do
  cp /tmp/fwa_$v.so $L
  timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-pcie --no-wire --no-wide $ARGS \
    > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}_${v}_$rep.log || { tail -5 gpurun_out/${TAG}_${v}_$rep.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${v}_$rep.json').read().strip().splitlines()[-1]); s=d['ingest_split_ms']; n=d['steps']; print('$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f fire %.3f' % (s['partition']/n, s['combine']/n, d['fire']['ms']/n))"
done; done
cp /tmp/fwa_a.so $L

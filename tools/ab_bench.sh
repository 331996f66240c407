#!/bin/bash
# Same-box A/B of library builds: bench.py with NIC_LIB pointing at each build in turn,
# ROUNDS interleaved passes (box-to-box variance exceeds most kernel deltas).
# usage: VARIANTS="cur=neural_network_image_compression_amd/libnic.so r1k=ab/libnic_r1k.so" bash tools/ab_bench.sh TAG
# a variant may add env settings after commas: "unfused=neural_network_image_compression_amd/libnic.so,NIC_K3P=0"
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${1:-ab}"; ROUNDS="${ROUNDS:-2}"; ARGS="${BENCH_ARGS:---steps 20 --warmup 3}"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARIANTS; do
    name="${v%%=*}"; spec="${v#*=}"; lib="${spec%%,*}"; envs=""
    [[ "$spec" == *,* ]] && envs="${spec#*,}"
    env ${envs//,/ } NIC_LIB="$ROOT/$lib" timeout -k 10 240 python bench.py $ARGS --no-cpu-baseline --no-parity \
      > "$OUT/${TAG}_${name}_$r.json" 2> "$OUT/${TAG}_${name}_$r.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$name] rc=$rc: stopping"; tail -5 "$OUT/${TAG}_${name}_$r.err"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], ' '.join(f\"{k}={v['avg_ms']:.4f}\" for k,v in d['layers'].items()))" \
      "$OUT/${TAG}_${name}_$r.json" "$name" "$r"
  done
done

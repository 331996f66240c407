#!/bin/bash
# round 6: same-box A/B of library builds (config 2, 3 alternating rounds; 4K once each)
# usage: bash tools/rounds/r6_ab.sh TAG v1 v2 ...   (v = base | suffix of libnic_<v>.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
B="--no-cpu-baseline --no-host-path --no-quality --no-power-probe --no-parity"
show() {
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], ' '.join(f\"{k}={v['avg_ms']:.4f}\" for k,v in d['layers'].items() if 'avg_ms' in v))" "$1" "$2"
}
for r in 1 2 3; do
  for v in "$@"; do
    lib=$PWD/neural_network_image_compression_amd/libnic_$v.so
    [ "$v" = base ] && lib=$PWD/neural_network_image_compression_amd/libnic.so
    NIC_LIB=$lib timeout -k 10 180 python bench.py --workload ${WL:-config2} --steps 30 --warmup 20 $B > $O/${v}_$r.json 2> $O/${v}_$r.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 $O/${v}_$r.err; exit $rc; }
    show $O/${v}_$r.json "$v/$r"
  done
done
[ "${NO4K:-0}" = 1 ] && exit 0
for v in "$@"; do
  lib=$PWD/neural_network_image_compression_amd/libnic_$v.so
  [ "$v" = base ] && lib=$PWD/neural_network_image_compression_amd/libnic.so
  NIC_LIB=$lib timeout -k 10 180 python bench.py --workload 4k --steps 10 --warmup 5 $B > $O/${v}_4k.json 2> $O/${v}_4k.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v 4k rc=$rc"; tail -5 $O/${v}_4k.err; exit $rc; }
  show $O/${v}_4k.json "$v/4k"
done

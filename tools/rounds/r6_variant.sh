#!/bin/bash
# round 6: parity subset of the GPU tests under NIC_LIB=libnic_<v>.so for each variant, then the
# same-box bench A/B (tools/rounds/r6_ab.sh) of base and the variants
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
K="${KEXPR:-encode_matches_golden or end_to_end or random_shapes or kodim21_full or 4k_frame or full_size_batch or encode_entropy_fold or batch_invariance}"
for v in ${PARITY:-$@}; do
  lib=$PWD/neural_network_image_compression_amd/libnic_$v.so
  [ "$v" = base ] && lib=$PWD/neural_network_image_compression_amd/libnic.so
  NIC_LIB=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_${v}_pytest.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/${TAG}_${v}_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/${TAG}_${v}_pytest.log | head -20; exit $rc; }
done
bash tools/rounds/r6_ab.sh $TAG base "$@"

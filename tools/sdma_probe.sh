env | grep -E "^(HSA_|GPU_|HIP_|ROC)" | sort
for v in "" "HSA_ENABLE_SDMA=1" "GPU_BLIT_ENGINE_TYPE=2" "GPU_BLIT_ENGINE_TYPE=1"; do
  echo "== $v"; env $v timeout -k 10 120 python tools/pcie_probe.py 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('ch3','ch4','h2d_12MB_ms','dev_dec_ms')})" || exit 1
done

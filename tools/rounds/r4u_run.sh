#!/bin/bash
# round 4: colour_split with 8 pixels / 16-B stores per thread (padded plane rows) vs 2 pixels
# (ab/libnic_cs2.so = the previous build) -- tests, kernel stats of both, interleaved bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "golden or encode or conv12 or c12 or trip" > $OUT/r4u_tests.log 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 $OUT/r4u_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 30 --warmup 10 --no-cpu-baseline --no-parity --no-power-probe --no-host-path --no-quality"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r4u_prof8 -o k -- python3 bench.py $B > $OUT/r4u_prof8.log 2>&1 || { echo "prof8 failed"; exit 1; }
NIC_LIB=$PWD/ab/libnic_cs2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r4u_prof2 -o k -- python3 bench.py $B > $OUT/r4u_prof2.log 2>&1 || { echo "prof2 failed"; exit 1; }
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > $OUT/r4u_c8_$r.json 2>/dev/null || { echo "c8 $r failed"; exit 1; }
  NIC_LIB=$PWD/ab/libnic_cs2.so timeout -k 10 200 python bench.py $B > $OUT/r4u_c2_$r.json 2>/dev/null || { echo "c2 $r failed"; exit 1; }
done
python3 - <<'PY'
import json, glob, csv
for t in ("c8_1","c2_1","c8_2","c2_2","c8_3","c2_3"):
    d=json.loads(open(f"gpurun_out/r4u_{t}.json").read().strip().splitlines()[-1])
    L=d["layers"]
    print(t, d["value"], d["ms_per_step"], {k: L[k].get("avg_ms") for k in ("conv2","conv8") if k in L})
for v in ("prof8","prof2"):
    for f in glob.glob(f"gpurun_out/r4u_{v}/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "colour_split" in row["Name"]:
                print(v, row["Calls"], row["AverageNs"])
PY
echo "[done]"

set -o pipefail
timeout -k 10 900 bash tools/profile.sh r03p_c5 --config c5 --cells 2000 --steps 6 --warmup 2 --no-cpu-baseline || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/prof_r03p_c5/summary.json"))
for k, v in d["kernels"].items():
    pm = v.get("pmc", {})
    print(k, v.get("median_ns"), {x: pm.get(x) for x in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
                                                         "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                                                         "SQ_INSTS_VALU_TRANS_F32", "SQ_WAVES")}, v.get("hbm_bytes_per_launch"))
PY

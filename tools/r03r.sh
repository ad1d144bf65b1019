set -o pipefail
timeout -k 10 600 bash tools/profile.sh r03r_s1 --fit step1 --steps 20 --warmup 3 --no-cpu-baseline || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/prof_r03r_s1/summary.json"))
for k, v in d["kernels"].items():
    pm = v.get("pmc", {})
    print(k, v.get("median_ns"), {x: pm.get(x) for x in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
                                                         "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU_TRANS_F32",
                                                         "SQ_WAVES")}, v.get("hbm_bytes_per_launch"))
PY

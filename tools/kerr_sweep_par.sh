#!/bin/bash
# The Kerr occlusion proof's envelope sweep (tools/kerr_proof_sweep.py) in 8 CPU processes with
# different seeds (CPU only: the restatement); records into gpurun_out/ksweep_<seed>.json.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for s in 11 12 13 14 15 16 17 18; do
  timeout -k 10 900 python3 tools/kerr_proof_sweep.py --configs 12 --rays 700 --seed $s --out gpurun_out/ksweep_$s.json > gpurun_out/ksweep_$s.log 2>&1 &
done
wait
python3 - <<'PY'
import json, glob
recs = []
for f in sorted(glob.glob("gpurun_out/ksweep_*.json")):
    recs += json.load(open(f))["records"]
out = dict(configs=len(recs), rays=sum(r["rays"] for r in recs), proven=sum(r["proven"] for r in recs),
           violations=sum(r["violations"] for r in recs),
           worst_deviation_over_delta=max(r["worst_deviation_over_delta"] for r in recs), records=recs)
json.dump(out, open("gpurun_out/ksweep_all.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "records"}))
PY

# predict_d2 A/B: north bench lines with the fused merged-grid whitening and with the distance pass +
# whiten_kfu_d2x2 in place, then the self-check against the C port with predict_d2=1.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04al
i=0
for s in "" "predict_d2=1" "" "predict_d2=1"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 --schedule "$s" > gpurun_out/r04al/b$i.json 2> gpurun_out/r04al/b$i.err || { tail -20 gpurun_out/r04al/b$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/r04al/b$i.json'));r=d['roofline_predict']
print('[$s]', round(d['ms_per_step'],1), round(r.get('wall_ms_per_step',0),1), {k:round(r[k]['avg_ms'],3) for k in ('pred_whiten','pred_adjoint','pred_var')})"
  i=$((i+1))
done
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --h2h-steps 0 --schedule predict_d2=1 > gpurun_out/r04al/check.json 2> gpurun_out/r04al/check.err || { tail -20 gpurun_out/r04al/check.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/r04al/check.json'));c=d['self_check']['cpu_port'];print({k:c[k] for k in ('dtc_rel','mean_max_abs','std_max_abs','mean_excess','std_excess','ok')})"

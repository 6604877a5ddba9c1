# round 5, sixteenth GPU batch: where the fused projection backward (rsx_linear_bwd, C5
# shape) spends its time -- timing ablations built by tools/build_variant.py: no dx
# products, no dW products, no sched_group_barrier orderings -- against the product build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b16}
mkdir -p $OUT
V=recommendar-systems_amd/rsx/lib/variants
for name in base lbwd_nodx lbwd_nodw lbwd_nosgb base; do
  if [ $name = base ]; then lib=""; else lib="RSX_LIB=$V/$name/librsx.so"; fi
  timeout -k 10 120 env $lib python tools/gpu/micro_gemm.py > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', round(d['rsx_linear_bwd_ms']*1e3,1), 'us')"
done
echo done

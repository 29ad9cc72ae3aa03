set -e
R=$GRAFT_REPO_ROOT
bash $R/scripts/pmc_attn.sh fwd
bash $R/scripts/pmc_attn.sh bwd --bwd
cd $R
for t in fwd bwd; do for p in a b c; do echo "== $t $p"; python3 scripts/pmc_summary.py $(find gpurun_out/pmc_${t}_${p} -name "*.db" | head -1) attn; done; done > gpurun_out/pmc_attn_summary.txt
cat gpurun_out/pmc_attn_summary.txt

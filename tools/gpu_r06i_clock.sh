# effective clock (GRBM_GUI_ACTIVE / 8 / wall) and MFMA-busy of the 25-kept rotation variants
set -o pipefail
for v in base rotg_w8d3 rotg_w8d3_diag5 rotg_off; do
  OPS=rotate_25 VARIANTS=$v NKV_PMC_PASSES="1 2" timeout -k 10 300 bash tools/gpu_pmc_kernels.sh r06i_$v > gpurun_out/r06i_$v.log 2>&1 || exit 1
done

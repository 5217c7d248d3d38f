# output_transform GEMM at M = 512 under tile / split overrides (tuning build), settled clock
#   bash tools/gemm_cfg_sweep.sh <tag>
set -e
tag=${1:-gcfg}
mkdir -p gpurun_out/$tag
run() { AZ_TUNING_LIB=1 "$@" timeout -k 10 120 python -u tools/gemm_ab.py 512,800 300 | sed "s/^/$(echo $@ | tr ' ' '_') /" >> gpurun_out/$tag/sweep.txt; }
run env
for s in 3 4 6 7 8; do run env AZ_GEMM_SPLITS=$s; done
for s in 2 3 4; do run env AZ_GEMM_X3=2 AZ_GEMM_SPLITS=$s; done
run env AZ_GEMM_X3=4

# conv2 study: hipBLASLt yardstick, the 8-phase kernel on dense shapes vs the tiled kernel, forward with/without conv12
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c2
mkdir -p $O
timeout -k 10 200 python3 tools/torch_gemm_ref.py > $O/torch.txt 2>&1 || exit 1; cat $O/torch.txt
timeout -k 10 200 python3 tools/op_driver.py gemm 10 11 ref4096s,conv2s > $O/t11.txt 2>&1 || exit 1; cat $O/t11.txt
CFM_GEMM8_DENSE=1 timeout -k 10 200 python3 tools/op_driver.py gemm 10 -1 ref4096s,conv2s > $O/g8.txt 2>&1 || exit 1; cat $O/g8.txt
CFM_CONV12=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/b_c0.json 2>> $O/err.txt || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/b_c1.json 2>> $O/err.txt || exit 1
python3 tools/show_bench.py $O/b_c0.json $O/b_c1.json | grep -E "==|conv|subsample"

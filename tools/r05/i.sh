set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i
mkdir -p $O
CFM_TN_CONV=0 timeout -k 10 200 python3 tools/tn_conv_check.py $O/g0.npz 2>> $O/err.txt || exit 1
CFM_TN_CONV=1 timeout -k 10 200 python3 tools/tn_conv_check.py $O/g1.npz 2>> $O/err.txt || exit 1
python3 tools/tn_conv_check.py --cmp $O/g1.npz $O/g0.npz
timeout -k 10 200 ./tools/lab/tn_lab 20 3 conv > $O/lab_conv.txt 2>&1 || exit 1
cat $O/lab_conv.txt
bash tools/env_train_ab.sh CFM_TN_CONV "0 1" 3
cat gpurun_out/ab_tests.log | tail -2

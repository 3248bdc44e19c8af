set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m
mkdir -p $O
for m in 0 1 2; do CFM_TN_CONV=$m timeout -k 10 200 python3 tools/tn_conv_check.py $O/g$m.npz 2>> $O/err.txt || exit 1; done
echo "mode 1 vs 0"; python3 tools/tn_conv_check.py --cmp $O/g1.npz $O/g0.npz
echo "mode 2 vs 0"; python3 tools/tn_conv_check.py --cmp $O/g2.npz $O/g0.npz
bash tools/env_train_ab.sh CFM_TN_CONV "1 2" 3
tail -1 gpurun_out/ab_tests.log

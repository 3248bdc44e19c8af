# same-box A/B: libcfm_base.so (HEAD~ sources) vs libcfm.so, interleaved, + stage breakdowns
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
bash tools/lib_ab.sh ${ROUNDS:-4} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
CFM_LIB_PATH=$PWD/conformer-nemo_amd/conformer_amd/libcfm_base.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/b_base.json 2>> $O/err.txt || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/b_new.json 2>> $O/err.txt || exit 1
python3 tools/show_bench.py $O/b_base.json $O/b_new.json

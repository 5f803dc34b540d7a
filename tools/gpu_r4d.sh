T=r4d VARIANTS="var_git_36b13f5 liblazydb_gpu var_def_LDB_LP2_0" ROUNDS=2 bash tools/gpu_session.sh || exit 1
VARIANTS="var_git_36b13f5 liblazydb_gpu var_def_LDB_LP2_0 var_def_LDB_WPB_12" CASES="3 w 1" ROUNDS=2 bash tools/scan_ab.sh

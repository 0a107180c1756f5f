cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BATCHES=6 CCRDT_LIB=$PWD/antidote_ccrdt_amd/lib/libccrdt_prof.so timeout -k 10 400 python tools/prof_resident.py > gpurun_out/tierR_phases_inplace.txt 2>&1; rc=$?; cat gpurun_out/tierR_phases_inplace.txt; exit $rc

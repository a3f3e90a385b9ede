set -o pipefail
cd $GRAFT_REPO_ROOT
GAMES=256 BLOCKS=6 FILTERS=64 bash tools/ab_run.sh gpurun_out/r05e_ab_novfc_c2.txt 800 $PWD/alphazero-chess_amd/azchess/libaz.so $PWD/abvar/novfc/libaz.so
cat gpurun_out/r05e_ab_novfc_c2.txt

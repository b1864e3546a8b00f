# GPU tests, then the config-3 and config-1 bench lines and their kernel-trace profiles
set -e
cd $GRAFT_REPO_ROOT
bash tools/_gpu_tests.sh
bash tools/_bench2.sh

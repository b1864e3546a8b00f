set -e
cd $GRAFT_REPO_ROOT
for a in 0 1 2 3 4 5; do
  KMP_BUCKET_ABLATE=$a timeout -k 10 120 python3 tools/time_engines.py 100000 5 residues 2>&1 | grep -E "stages|median" | sed "s/^/abl=$a /" | cut -c1-200
done

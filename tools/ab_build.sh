# builds tools/ab/<name>/libkmerpair.so: the library with kmp_postings.hip compiled with extra flags
#   bash tools/ab_build.sh NAME -DFOO=1 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../uniprot_kmer_based_clustering_amd/csrc"
mkdir -p ../../tools/ab/$name
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. -w "$@" -c kmp_postings.hip -o /tmp/kmp_postings_$name.o
objs=$(ls ../build/*.o | grep -v '/kmp_postings.o')
hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/$name/libkmerpair.so $objs /tmp/kmp_postings_$name.o -ldl -lpthread
echo built tools/ab/$name

# build libkmerpair variants of kmp_postings.hip (name:flags pairs) into build_variants/
set -e
cd "$(dirname "$0")/../uniprot_kmer_based_clustering_amd/csrc"
make -s -j8
mkdir -p ../../build_variants
OBJS=$(ls ../build/*.o | grep -v kmp_postings.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-result $flags \
    -c kmp_postings.hip -o ../../build_variants/kmp_postings_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build_variants/libkmerpair_$name.so $OBJS ../../build_variants/kmp_postings_$name.o
done
rm -f ../../build_variants/*.o
ls ../../build_variants/*.so

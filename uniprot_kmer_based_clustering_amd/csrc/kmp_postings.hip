// kmp_postings.hip — the postings engine: the reference's own pair algorithm restated for the
// GPU as sort / expand / reduce.
//
//   reference (file:line)                                  here
//   Protein::new windows + codes (protein.rs:82-94)        residue_keys_chunk_kernel: one key per window
//   per-protein sort + dedup (main.rs:99-101,187-189)             duplicates of (k-mer, p) end up adjacent
//                                                          after the stable code sort; skipped there
//   global df: sorted Vec<(kmer, df)> (main.rs:77-122)     radix sort of the keys on the code bits;
//                                                          one run per distinct k-mer, df = distinct
//                                                          proteins in the run
//   repeat split df >= 2 (main.rs:127-149)                 runs with df >= 2
//   Graph::new: C(df,2) KmerEdge::Single per k-mer         expand_kernel: every (k-mer, p, q) incidence
//     (graph/mod.rs:39-193, vertex.rs:59-140)                of a run, one thread per run element
//   remove_uninteresting_edges (mod.rs:549-697)            class test fused into the expansion
//   combine_edges: Group per pair, len = w (mod.rs:322-546) radix sort of pair keys p*N+q, run-length
//                                                          encode: run length = w; the runs come out in
//                                                          canonical (p, q) order
// Work is O(Σ C(df,2)) like the reference (no N² scan).
//
// Key layout (u64): [ code | class (16 bits, when it fits) | p (pbits) ].  Only the code bits are
// sorted; the sort is stable and keys are laid out in protein order, so every run lists its
// proteins ascending.  Carrying the class in the key keeps the expansion free of random loads.
#include <hip/hip_runtime.h>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <chrono>
#include <memory>
#include <vector>

#include "kmerpair.h"
#include "kmp_internal.hpp"

using namespace kmp;

// The engine is one translation unit, included stage by stage from postings/ (each file is
// only meaningful inside this one: shared internal types, kernels and templates).
namespace {
#include "postings/keys.hip"
#include "postings/group.hip"
#include "postings/heavy.hip"
#include "postings/partition.hip"
}  // namespace
#include "postings/workspace.hip"
namespace {
#include "postings/front.hip"
#include "postings/tail.hip"
#include "postings/tail_multi.hip"
#include "postings/step.hip"
#include "postings/split.hip"
}  // namespace
#include "postings/api.hip"

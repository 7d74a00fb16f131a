// rs_inst.hip — the kernel instances of one source-column count K.
//
// Compiled once per K = 1..16 with -DELECT_EC_INST_K=K (elect_amd/build.py),
// so the launchers and kernels of every (K, R = 1..4) shape build in parallel
// translation units; rs_kernels.hip's dispatch table reaches them through
// kernel_rows_kK().
#include "rs_impl.hpp"

#ifndef ELECT_EC_INST_K
#error "compile rs_inst.hip with -DELECT_EC_INST_K=<source columns, 1..16>"
#endif
static_assert(ELECT_EC_INST_K >= 1 && ELECT_EC_INST_K <= elect::kern::kMaxCols, "ELECT_EC_INST_K out of range");

#define ELECT_EC_CAT2(a, b) a##b
#define ELECT_EC_CAT(a, b) ELECT_EC_CAT2(a, b)

namespace elect {
namespace kern {

KernelRows ELECT_EC_CAT(kernel_rows_k, ELECT_EC_INST_K)()
{
    constexpr int K = ELECT_EC_INST_K;
    KernelRows r;
    r.fast = fast_row_fns<K>();
    if constexpr (K <= kMaxPadCols) r.pad = fast_row_fns<K, true>();
    r.group = group_row_fns<K>();
    return r;
}

}  // namespace kern
}  // namespace elect

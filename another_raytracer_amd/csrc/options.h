// options.h — process-wide library options (rt_option_set / rt_option_get, include/art.h).
//
// Everything that used to be an environment knob lives here, set only by an explicit call: the scene compiler's
// experiment switches (world merging, hoisting, the BVH builder's SAH parameters and collapse), the upload's 16-bit
// child codes, the multi-GPU deadline and the test fault points.  Nothing is read from the environment, except that
// multi.timeout_ms falls back to the documented ART_MULTI_TIMEOUT_MS when it was never set.  A stray variable in an
// embedding application's environment can therefore neither inject a fault nor change a tree.
#pragma once
#include <cstddef>

namespace art {

enum class Opt : int {
    // scene compile (applies to scenes compiled after the call)
    WorldMerge,    // compile.world_merge: 0 off, 1 BVH runs only, 2 (default) BVH runs and primitive runs
    Hoist,         // compile.hoist: 1 (default) hoist large primitives out of their BVH, 0 off
    BvhCollapse,   // bvh.collapse: 0 (default) greedy 4-wide collapse, 1 SAH-optimal dynamic programme
    CollapseCi,    // bvh.collapse_ci: the DP collapse's primitive-test cost per 4-wide node visit (0.6)
    DpBinaryLeaf,  // bvh.dp_binary_leaf: binary-tree leaf size under the DP collapse (1)
    SahCi,         // bvh.sah_ci: SAH primitive-test cost per binary node step (1.5)
    SahLeaf,       // bvh.sah_leaf: largest leaf (4)
    Sbvh,          // bvh.sbvh: spatial-split reference budget (1.5; < 1 turns spatial splits off)
    SbvhAlpha,     // bvh.sbvh_alpha: overlap / root area below which no spatial split is tried (1e-5)
    // device upload and launch (applies to uploads / renders after the call)
    Codes16,       // render.codes16: 1 (default) 16-bit child codes where they fit, 0 always the 32-bit-code kernels
    LdsNodesMax,   // render.lds_nodes_max: cap on the LDS-resident nodes of a partial-LDS (LM 2) kernel (diagnostic)
    Leaf2,         // render.leaf2: 1 (default) pair-aligned leaves where 16-bit codes need them (F_LEAF2), 0 off
    TexBary,       // render.tex_bary: 1 (default) the TF_BARY kernels for meshes whose only images are barycentric, 0 off
    // multi-GPU
    MultiTimeoutMs,  // multi.timeout_ms: deadline of RCCL init / gather waits (unset: ART_MULTI_TIMEOUT_MS, else 120000;
                     // inf, or anything beyond ~292 years, means no deadline)
    RcclBlocking,    // multi.rccl_blocking: 1 = blocking communicators (diagnosis), 0 (default) non-blocking.  Blocking
                     // gives up the deadline and the error-path protection: an error between the communicator inits
                     // (before every rank is issued) leaves the group's ncclGroupEnd waiting for ranks never issued
    // test fault points (tests only: each makes a specific later call fail as the real fault would)
    FaultWorkspaceBytes,  // test.fault_workspace_bytes: refuse workspace growth beyond this many bytes (0 = off)
    FaultGatherAbort,     // test.fault_gather_abort: 1 = the next rt_render_multi's gather fails in flight
    FaultRcclGroup,       // test.fault_rccl_group: 1 = rt_multi_create / 2 = rt_render_multi throws inside its RCCL group
    kCount
};

// The option's current value (its default unless set).  MultiTimeoutMs: see above.
double opt(Opt o);
// By name; false for an unknown name or a value outside the option's range (why says which).
bool opt_set(const char* name, double value, const char** why);
bool opt_get(const char* name, double* value);
void opt_reset_all();

}  // namespace art

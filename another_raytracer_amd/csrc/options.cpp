// options.cpp — the option table behind rt_option_set / rt_option_get (options.h).
#include "options.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>

namespace art {

namespace {

struct OptDef {
    const char* name;
    double def, lo, hi;
    bool integer;
};
constexpr double kInf = std::numeric_limits<double>::infinity();
// index = Opt value
const OptDef kDefs[static_cast<int>(Opt::kCount)] = {
    {"compile.world_merge", 2, 0, 2, true},
    {"compile.hoist", 1, 0, 1, true},
    {"bvh.collapse", 0, 0, 1, true},
    {"bvh.collapse_ci", 0.6, 0, 1e6, false},
    {"bvh.dp_binary_leaf", 1, 1, 16, true},
    {"bvh.sah_ci", 1.5, 0, 1e6, false},
    {"bvh.sah_leaf", 4, 1, 16, true},
    {"bvh.sbvh", 1.5, 0, 1e6, false},
    {"bvh.sbvh_alpha", 1e-5, 0, 1e6, false},
    {"render.codes16", 1, 0, 1, true},
    {"render.lds_nodes_max", 4294967295.0, 0, 4294967295.0, true},
    {"render.leaf2", 1, 0, 1, true},
    {"render.tex_bary", 1, 0, 1, true},
    {"multi.timeout_ms", std::numeric_limits<double>::quiet_NaN(), 0, kInf, false},
    {"multi.rccl_blocking", 0, 0, 1, true},
    {"test.fault_workspace_bytes", 0, 0, 1.8e19, true},
    {"test.fault_gather_abort", 0, 0, 1, true},
    {"test.fault_rccl_group", 0, 0, 2, true},
};

std::atomic<double> g_val[static_cast<int>(Opt::kCount)];
std::atomic<bool> g_init{false};

void init_once() {
    if (g_init.load(std::memory_order_acquire)) return;
    static const bool done = [] {
        opt_reset_all();
        g_init.store(true, std::memory_order_release);
        return true;
    }();
    (void)done;
}

int find(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < static_cast<int>(Opt::kCount); ++i)
        if (std::strcmp(kDefs[i].name, name) == 0) return i;
    return -1;
}

}  // namespace

void opt_reset_all() {
    for (int i = 0; i < static_cast<int>(Opt::kCount); ++i) g_val[i].store(kDefs[i].def, std::memory_order_relaxed);
}

double opt(Opt o) {
    init_once();
    const double v = g_val[static_cast<int>(o)].load(std::memory_order_relaxed);
    if (o == Opt::MultiTimeoutMs && std::isnan(v)) {  // never set: the documented environment default
        const char* s = std::getenv("ART_MULTI_TIMEOUT_MS");
        return (!s || !*s) ? 120000.0 : std::max(0.0, std::strtod(s, nullptr));
    }
    return v;
}

bool opt_set(const char* name, double value, const char** why) {
    init_once();
    const int i = find(name);
    if (i < 0) {
        *why = "unknown option";
        return false;
    }
    const OptDef& d = kDefs[i];
    if (!(value >= d.lo && value <= d.hi) || (d.integer && value != std::floor(value))) {
        *why = d.integer ? "value outside the option's integer range" : "value outside the option's range";
        return false;
    }
    g_val[i].store(value, std::memory_order_relaxed);
    return true;
}

bool opt_get(const char* name, double* value) {
    init_once();
    const int i = find(name);
    if (i < 0) return false;
    *value = opt(static_cast<Opt>(i));
    return true;
}

}  // namespace art

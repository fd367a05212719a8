// MI355X GAT library: ABI version, table layout and the A/B knob snapshot.

#include "gat_common.h"

namespace gat_detail __attribute__((visibility("hidden"))) {

// Kernel-choice knobs for A/B measurement (tools/, tests; not part of the
// ABI).  The environment is read ONCE, at the first launch, into a snapshot;
// gat_tuning_reload() re-reads it (for the tools and tests that switch
// variants within one process).  The specialised kernels are the default
// wherever the shape allows them.
static const char* const kKnobNames[] = {
    "GAT_PROJ_KERNEL", "GAT_PROJ_WK_MAX", "GAT_EDGE_LDS",  "GAT_EDGE_V",   "GAT_EDGE_U",
    "GAT_EDGE_PIPE",   "GAT_EDGE_SCORE",  "GAT_EDGE_KERNEL", "GAT_BWD_LDS", "GAT_BWD_U",
    "GAT_BWD_KERNEL",  "GAT_BWD_WAVES",   "GAT_HUB_SEG",     "GAT_PROJ_X3",
    "GAT_PROJ_BM",     "GAT_PROJ_WRES",   "GAT_PROJ_WRES_WGS", "GAT_BWD_KINK",
    "GAT_WGRAD_LW",    "GAT_STORE_WT",    "GAT_PROJ_WK_DIRECT", "GAT_EDGE_SPLIT",
    "GAT_PROJ_X3V",    "GAT_PROJ_WG",     "GAT_EDGE_LDSDMA", "GAT_PROJ_PRESPLIT", "GAT_BWD_SL",
    "GAT_EDGE_HL",     "GAT_PROJ_WRES_DIRECT", "GAT_EDGE_XPROJ", "GAT_EDGE_MERGE", "GAT_EDGE_ROWCOL"};
constexpr int kNumKnobs = (int)(sizeof(kKnobNames) / sizeof(kKnobNames[0]));

struct KnobSnapshot {
    bool set[kNumKnobs];
    char val[kNumKnobs][32];
};
static KnobSnapshot g_knobs;
static bool g_knobs_ready = false;

void snapshot_knobs() {
    for (int i = 0; i < kNumKnobs; ++i) {
        const char* v = std::getenv(kKnobNames[i]);
        g_knobs.set[i] = v != nullptr;
        g_knobs.val[i][0] = '\0';
        if (v != nullptr) {
            std::strncpy(g_knobs.val[i], v, sizeof(g_knobs.val[i]) - 1);
            g_knobs.val[i][sizeof(g_knobs.val[i]) - 1] = '\0';
        }
    }
    g_knobs_ready = true;
}

const char* knob(const char* name) {
    if (!g_knobs_ready) snapshot_knobs();
    for (int i = 0; i < kNumKnobs; ++i)
        if (std::strcmp(kKnobNames[i], name) == 0) return g_knobs.set[i] ? g_knobs.val[i] : nullptr;
    return nullptr;
}

int store_wt_on() {
    const char* v = knob("GAT_STORE_WT");
    return v != nullptr ? std::max(0, std::min(3, std::atoi(v))) : 1;
}

bool kernel_choice(const char* env, const char* slow) {
    const char* v = knob(env);
    return !(v != nullptr && std::strcmp(v, slow) == 0);
}

}  // namespace gat_detail

extern "C" {

int gat_abi_version(void) { return GAT_ABI_VERSION; }

int gat_tuning_reload(void) {
    snapshot_knobs();
    return GAT_OK;
}

int gat_table_layout(int heads, int f, int* ld, int* s_off) {
    if (heads <= 0 || f <= 0 || ld == nullptr || s_off == nullptr) return GAT_EINVAL;
    const int hf = heads * f;
    *s_off = round_up4(hf);
    *ld = *s_off + round_up4(heads);
    return GAT_OK;
}

}  // extern "C"

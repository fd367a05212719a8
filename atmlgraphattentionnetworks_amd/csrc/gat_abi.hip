// MI355X GAT library: ABI version, table layout and the knob snapshot.

#include "gat_common.h"

namespace gat_detail __attribute__((visibility("hidden"))) {

// Kernel-choice knobs (not part of the ABI): each forces one of two product
// paths that a shape or a graph can also reach, so that the tests can compare
// them on one input (bitwise where the arithmetic is the same).  The
// environment is read ONCE, at the first launch, into a snapshot;
// gat_tuning_reload() re-reads it (for the tests that switch paths within one
// process).  The defaults are the measured-fastest choices; the round-1..5
// A/B knobs whose losing arms are recorded under profiles/ were removed with
// their kernels in round 6.
static const char* const kKnobNames[] = {
    "GAT_EDGE_U",      // edges per chunk: 4, 8 or 16 (default by edges per row)
    "GAT_EDGE_V",      // float4s per lane: 1 or 2 (default by edges per row)
    "GAT_EDGE_PIPE",   // 0: the U = 16, V = 2 kernel without gathers one chunk ahead
    "GAT_EDGE_SPLIT",  // lane groups per row: 1, 2 or 4 (default by launch size)
    "GAT_EDGE_ROWCOL", // 0: short-row col values one chunk ahead, not 8 per load
    "GAT_EDGE_XPROJ",  // 0: Fin <= 4 as projection + edge kernel, not fused
    "GAT_BWD_KINK",    // 0: the backward's target pass over the edges, not the kink sums
    "GAT_BWD_SL",      // 0: the generic source pass, not the straight-line HF = 64 one
    "GAT_BWD_KERNEL",  // stored | generic: the stored-coefficient backward
};
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

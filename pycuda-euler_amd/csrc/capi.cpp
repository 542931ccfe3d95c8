// capi.cpp -- error state and version of the libeulerhip C ABI (include/eulerhip.h).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace ec {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

static thread_local Knobs g_knobs;
const Knobs &kn() { return g_knobs; }
void refresh_knobs() {
    Knobs k;
    if (getenv("EULERHIP_DEBUG")) {
        auto flag = [](const char *n) { return getenv(n) != nullptr; };
        auto num = [](const char *n, int dflt) {
            const char *e = getenv(n);
            return e ? atoi(e) : dflt;
        };
        k.no_sk2 = flag("EULERHIP_NO_SK2");
        k.no_v2 = flag("EULERHIP_NO_V2");
        k.force_filter = flag("EULERHIP_FORCE_FILTER");
        k.no_filter = flag("EULERHIP_NO_FILTER");
        k.filter_pmax = num("EULERHIP_FILTER_PMAX", 0);
        k.filter_pmin = num("EULERHIP_FILTER_PMIN", -1);
        if (const char *e = getenv("EULERHIP_PART_KEYS")) k.part_keys = (float)atof(e);
        k.v2_r10 = num("EULERHIP_V2_R10", -1);
        k.refine_rs = num("EULERHIP_REFINE_RS", 0);
        k.no_spec = num("EULERHIP_NO_SPEC", 0);
        k.tile_plan = num("EULERHIP_TILE_PLAN", -1);
        k.rj_div = num("EULERHIP_RJ_DIV", 0);
        k.rank_sync = num("EULERHIP_RANK_SYNC", 0);
        k.merge_mix = flag("EULERHIP_MERGE_MIX");
        k.merge_decode = flag("EULERHIP_MERGE_DECODE");
        k.skf_merge = num("EULERHIP_SKF_MERGE", 1);
        k.wide_runs = num("EULERHIP_WIDE_RUNS", 1);
        k.no_small_starts = flag("EULERHIP_NO_SMALL_STARTS");
        k.wide_general = flag("EULERHIP_WIDE_GENERAL");
        k.wide_max_bbits = num("EULERHIP_WIDE_MAX_BBITS", -1);
        k.wide_l3 = num("EULERHIP_WIDE_L3", 0);
        k.join_links = num("EULERHIP_JOIN_LINKS", -1);
        k.join_cap = num("EULERHIP_JOIN_CAP", 0);
        k.junction_bt = num("EULERHIP_JUNCTION_BT", -1);
        k.sk2_elim = num("EULERHIP_SK2_ELIM", 0);
        k.no_char_pack = num("EULERHIP_NO_CHAR_PACK", 0);
        k.wr_one = num("EULERHIP_WR_ONE", 0);
        k.junction_sb = num("EULERHIP_JUNCTION_SB", 0);
        k.junction_claim = num("EULERHIP_JUNCTION_CLAIM", 0);
        if (const char *e = getenv("EULERHIP_WIDE_L3_CAP")) k.wide_l3_cap = atoll(e);
        k.host_chunks = num("EULERHIP_HOST_CHUNKS", 0);
        k.sk2_stats = flag("EULERHIP_SK2_STATS");
        k.no_slot_groups = flag("EULERHIP_NO_SLOT_GROUPS");
        k.no_skb3 = flag("EULERHIP_NO_SKB3");
        k.sk2_claim = num("EULERHIP_SK2_CLAIM", 0);
        k.verbose = flag("EULERHIP_VERBOSE");
        k.rank = num("EULERHIP_RANK", -1);
        k.sk_filt = num("EULERHIP_SK_FILT", -1);
        k.skf_keys = num("EULERHIP_SKF_KEYS", 0);
        k.wide_mb = num("EULERHIP_WIDE_MB", -1);
        k.join_mb = num("EULERHIP_JOIN_MB", -1);
        k.join_local = num("EULERHIP_JOIN_LOCAL", -1);
        k.junction_radix = num("EULERHIP_JUNCTION_RADIX", -1);
        k.copy_streams = num("EULERHIP_COPY_STREAMS", -1);
        k.run_packed = num("EULERHIP_RUN_PACKED", -1);
        k.upsweep_staged = num("EULERHIP_UPSWEEP_STAGED", -1);
        k.jl_fcap = num("EULERHIP_JL_FCAP", -1);
        k.jl_bits_delta = num("EULERHIP_JL_BITS_DELTA", 0);
        k.sruler_mask = num("EULERHIP_SRULER_MASK", 0);
    }
    g_knobs = k;
}
bool memlog_on() {
    static const bool on = getenv("EULERHIP_MEMLOG") != nullptr;
    return on;
}
}  // namespace ec

extern "C" const char *ec_last_error(void) { return ec::g_err; }
extern "C" int ec_version(void) { return 100; /* 0.1.0 */ }

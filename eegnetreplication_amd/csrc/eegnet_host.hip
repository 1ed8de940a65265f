// eegnet_host.hip -- host side of libeegnet_hip.so: geometry/validation, workspace layout, launch
// sequences of the train step and the C-ABI of include/eegnet_abi.h.  Included by eegnet_kernels.hip.
// ================================================================================================
// Host side: geometry, validation, launch sequences, C-ABI.
// ================================================================================================
using namespace eeg;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// dynamic LDS per workgroup: 160 KiB less a little room for the static LDS of the traced build
constexpr int LDS_MAX = 160 * 1024 - 256;

static inline int rup(int a, int m) { return (a + m - 1) / m * m; }
static inline size_t rupz(size_t a, size_t m) { return (a + m - 1) / m * m; }

constexpr size_t CNT_BYTES = (size_t)TK_COUNT * NCNT * 4;     // 800 B, a multiple of 16

struct WsLayout {
    size_t cnt, partA, partB, partC, partD, partE, sums, stats, coef, d2, E1, E2, dp2, dl, s, v, q3, r3;
    size_t total;
};

static int device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;     // MI355X
    }
    return cus;
}

static unsigned long long* g_trace_buf = nullptr;     // eegnet_trace_enable

static int make_geo_wide(Geo* g, bool launch);

// LDS (floats) of the whole-trial block-2 passes (eegnet_wide.hip k_wpass_b2 / c / d) at nw waves
static void b2_lds(Geo* g, int nw) {
    auto tailw = [](int ncols, int fin) { return 2 * (tail_s_doubles(ncols) + fin); };
    const int nf4 = (g->NF + 3) / 4 * 4;
    const int b2 = 2 * g->F2P * g->RB + g->F2P * K2 + g->F2P * (g->F2P + 1);   // D2, Q, w2, W3 tables
    const int TQ1 = (g->T1 + 3) / 4;
    g->ldsWB2 = std::max(b2 + nw * 2 * 16, tailw(g->nB, 0));
    g->ldsWC = std::max(nf4 + nw * 4 + nw * 2 * 16 + g->F2P * g->RB, tailw(g->nC, 0));    // H | sums | XH
    g->ldsWD = std::max(b2 + g->F2P * g->RB + nf4 + 2 * g->F2 * TQ1, tailw(g->nD, 0));
}

// Launch-shape choices fixed at build time (the shipped library reads no environment: kernel choice and
// grids are functions of the dims alone).  A/B experiments build variants with -D (tools/ab.sh).
//
// Block-2 passes C / D of the F2 <= 16 step: one trial per wave (k_pass_c / k_pass_d, the default)
// or whole-trial 256-thread workgroups (the wide path's k_wpass_c / k_wpass_d, -DEEGNET_B2=1).  Before
// pass B stored the q / r planes the whole-trial kernels won at small per-launch grids (batch 64,
// fold-indexed launches); with the planes the one-trial-per-wave kernels win the fold-indexed
// real-protocol leg (6.5 M against 5.9 M trials/s) and lose 3-7% on a lone batch of 64.  One rule
// for every launch keeps a fold-indexed step bit-identical to the same fold's FusedTrainer step.
#ifndef EEGNET_B2
#define EEGNET_B2 0
#endif
static bool use_b2_narrow(const Geo&) { return EEGNET_B2 == 1; }

// Pass D of the F2 <= 16 step: the row-layout kernel k_pass_dr (two 512-thread workgroups per CU on the
// streaming grid, the workgroup on one trial at a time; eegnet_passes.hip), or -DEEGNET_D1=1 the
// one-trial-per-wave k_pass_d of rounds 1-5 (A/B builds)
#ifndef EEGNET_D1
#define EEGNET_D1 0
#endif

// workgroups per CU slot of the streaming passes A / B / E (-DEEGNET_GRIDS_MULT=n, experiments): with
// more workgroups than resident slots the dispatcher refills a CU's early-finishing slot, so the two
// resident workgroups' skew turns into load balance; the same for passes C / D (-DEEGNET_GRIDC_MULT)
#ifndef EEGNET_GRIDS_MULT
#define EEGNET_GRIDS_MULT 1
#endif
#ifndef EEGNET_GRIDC_MULT
#define EEGNET_GRIDC_MULT 1
#endif
static_assert(EEGNET_GRIDS_MULT >= 1 && EEGNET_GRIDS_MULT <= 8 && EEGNET_GRIDC_MULT >= 1 && EEGNET_GRIDC_MULT <= 8,
              "grid multipliers are 1..8");
static constexpr int grid_mult() { return EEGNET_GRIDS_MULT; }
static constexpr int grid_mult_cd() { return EEGNET_GRIDC_MULT; }

// the compile-time shape of the narrow passes (EEG_DISPATCH) whose x loads honour a row pitch: 22 x 257
// (the recordings), whose 257-float rows are not 16-byte units; 22 x 256 rows already are, and its
// kernels take the pitch as the compile-time T (EEG_XP)
static bool x_pitch_shape(const eegnet_dims& d) {
    return d.K1 == 32 && d.C == 22 && d.T == 257 && d.F1 == 8 && d.D == 2;
}

static int make_geo(const eegnet_dims* d, Geo* g, bool launch = true) {
    if (!d) return fail(EEGNET_EINVAL, "dims is NULL");
    memset(g, 0, sizeof(*g));
    g->trace = g_trace_buf;
    g->B = d->B; g->C = d->C; g->T = d->T; g->F1 = d->F1; g->D = d->D; g->K1 = d->K1;
    g->Bn = d->B;
    g->F2 = d->F1 * d->D;
    if (g->B < 1) return fail(EEGNET_EINVAL, "B must be >= 1 (got %d)", g->B);
    if (g->K1 != 32 && g->K1 != 64) return fail(EEGNET_EINVAL, "K1 must be 32 or 64 (got %d)", g->K1);
    if (g->C < 1 || g->C > 64) return fail(EEGNET_EINVAL, "C must be in [1,64] (got %d)", g->C);
    if (g->F1 < 1 || g->D < 1 || g->F2 > 64 || (g->F2 & 3))
        return fail(EEGNET_EINVAL, "F1*D must be a multiple of 4 in [4,64] (got F1=%d D=%d)", g->F1, g->D);
    if (g->T < 32 || g->T < g->K1 || g->T > 1024)
        return fail(EEGNET_EINVAL, "T must be in [max(32,K1), 1024] (got %d)", g->T);
    g->XP = d->x_pitch ? d->x_pitch : g->T;
    if (g->XP != g->T && !(x_pitch_shape(*d) && (g->XP & 3) == 0 && g->XP > g->T))
        return fail(EEGNET_EINVAL, "x_pitch %d: only the 22 x 257 EEGNet-8,2 (K1 = 32) training kernels take "
                    "a row pitch, a multiple of 4 above T (eegnet_x_pitch)", g->XP);
    g->P = (g->K1 - 1) / 2; g->R = g->K1 - 1 - g->P;
    g->T1 = g->T / 4; g->T2 = g->T1 / 8; g->NF = g->F2 * g->T2;
    g->LP = (g->R + 3) & ~3;
    g->TQ = (g->T + 3) / 4; g->NT16 = (g->T + 15) / 16; g->NKG = g->NT16;
    g->RS = row_stride(g->K1, g->T);
    g->RS2 = rup(LP2 + g->T1 + 8, 4);
    g->CK = rup(g->C, 4); g->NCT = (g->C + 15) / 16;
    g->nH = g->R * (g->R + 1) / 2;
    g->nTl = g->P * (g->P + 1) / 2;
    g->nedge = g->nH + g->nTl + g->R + g->P;
    g->p = d->p_drop; g->eps = d->bn_eps; g->mom = d->bn_momentum;
    if (!(g->p >= 0.f && g->p <= 1.f)) return fail(EEGNET_EINVAL, "p_drop must be in [0,1]");
    g->scale = g->p < 1.f ? 1.f / (1.f - g->p) : 0.f;
    int o = 0;
    g->o_w1 = o; o += g->F1 * g->K1;
    g->o_g1 = o; o += g->F1;
    g->o_b1 = o; o += g->F1;
    g->o_ws = o; o += g->F2 * g->C;
    g->o_g2 = o; o += g->F2;
    g->o_b2 = o; o += g->F2;
    g->o_w2 = o; o += g->F2 * 16;
    g->o_W3 = o; o += g->F2 * g->F2;
    g->o_g3 = o; o += g->F2;
    g->o_b3 = o; o += g->F2;
    g->o_Wfc = o; o += NCLS * g->NF;
    g->o_bfc = o; o += NCLS;
    g->nparam = o;
    if (g->NF < 1) return fail(EEGNET_EINVAL, "T//32 must be >= 1");
    g->nA = g->K1 + 1 + g->nedge + 2 * g->F2;
    g->nB = 2 * g->F2;
    g->nC = NCLS * g->NF + NCLS + 2 * g->F2 + 1;
    g->nD = g->F2 * g->F2 + 18 * g->F2;
    g->QR = (g->F2 <= F2MAX && g->D == 2) ? g->F1 : g->F2;
    g->nE = g->QR * g->K1 + g->F2 * g->C + 2 * g->F2;
    g->grid = std::min(g->B, device_cus() * grid_mult_cd());     // passes C, D, infer
    g->gridS = std::min(g->B, device_cus() * WGPC * grid_mult());     // streaming passes A, B, D, E
    g->gridA = g->gridE = g->gridS;
    const int rows1 = g->C * g->RS;                   // x rows (one buffer)
    const int nf4 = rup(g->NF, 4);
    const bool spec = g->C == 22 && (g->T == 256 || g->T == 257) && g->F1 == 8 && g->D == 2 && g->K1 == 32;   // EEG_DISPATCH
    // compile-time shapes: two x buffers, and two xstat-row slots (fold launches, eegnet_fold.xstat)
    g->ldsA = (spec ? 2 : 1) * rows1 + g->F2 * g->RS + NWB * (g->K1 + 1) + (spec ? 2 * rup(g->K1 + 1 + g->nedge, 4) : 0);
    g->ldsB = 3 * g->F2 * g->RS2 + F2MAX * (K2 + F2MAX);
    // passes C / D: one trial stream per wave, each with its own block-2 rows (row_stride_b2)
    g->RSW = row_stride_b2(g->T1);
    const int pwC = nf4, pwD = 3 * g->F2 * g->RSW + nf4;
    g->nwC = std::max(1, std::min(spec ? NWAVE : NTHS / 64, (LDS_MAX / 4 - 4 * F2MAX) / pwC));
    g->nwD = std::max(1, std::min(NTHS / 64, (LDS_MAX / 4) / pwD));
    g->ldsC = std::max(g->nwC * pwC + 4 * F2MAX, g->nwC * g->nC);   // Hs rows + the BN3 constant table
    g->ldsD = EEGNET_D1 ? std::max(g->nwD * pwD, g->nwD * g->nD)
                        : std::max(dr_lds_floats(spec ? 1 : MAXT1Q), dr_tail_floats(spec));
    g->ldsE = std::max((2 * g->F2 + g->C) * g->RS + rup(g->F2 * g->T1, 4) + 8 * g->F2,
                       NWB * 256 * (1 + (15 + g->K1 - 1) / 16 + 1));   // after the loop: dws, Cq tiles
    g->ldsI = rows1 + g->F2 * g->RS + 2 * g->F2 * g->RS2 + nf4;
    // the reduction tail and finalize reuse each pass kernel's LDS (doubles = 2 floats)
    auto tail = [](int ncols, int fin) { return 2 * (tail_s_doubles(ncols) + std::max(tail_scratch_doubles(ncols), fin)); };
    g->ldsA = std::max(g->ldsA, tail(g->nA, fin1_scratch_doubles(g->K1, g->F1, g->F2, g->C)));
    g->ldsB = std::max(g->ldsB, tail(g->nB, 0));
    g->ldsC = std::max(g->ldsC, tail(g->nC, 0));
    g->ldsD = std::max(g->ldsD, tail(g->nD, 0));
    g->ldsE = std::max(g->ldsE, tail(g->nE, fin5_scratch_doubles(g->K1, g->F1, g->o_g2)));
    g->wide = g->F2 > F2MAX ? 1 : 0;
    if (g->wide) return make_geo_wide(g, launch);
    g->F2P = 16;
    g->RB = rb_stride(g->T1);
    b2_lds(g, 4);
    g->gridB2 = std::min(g->B, 4 * device_cus());
    if (launch) {
        if (g->C * g->T > NTH * MAXPF)
            return fail(EEGNET_EINVAL, "C*T = %d exceeds the %d-float prefetch of one trial", g->C * g->T,
                        NTH * MAXPF);
        if (g->T1 > 64 * MAXT1Q) return fail(EEGNET_EINVAL, "T/4 > %d", 64 * MAXT1Q);
        if (g->F2 * g->T1 > 4 * NTH) return fail(EEGNET_EINVAL, "F2*(T/4) > %d", 4 * NTH);
        if ((double)g->B * g->F2 * g->T1 >= 4294967296.0)
            return fail(EEGNET_EINVAL, "B*F2*(T/4) must stay below 2^32 (dropout / mask indices)");
        if (g->NF > 64 * MAXNFQ) return fail(EEGNET_EINVAL, "F2*(T/32) = %d > %d", g->NF, 64 * MAXNFQ);
        if (g->nparam > APT * NTB) return fail(EEGNET_EINVAL, "%d parameters > %d", g->nparam, APT * NTB);
        const int lmax = std::max(std::max(std::max(g->ldsA, g->ldsB), std::max(g->ldsC, g->ldsD)),
                                  std::max(g->ldsE, g->ldsI));
        if (lmax * 4 > LDS_MAX) return fail(EEGNET_EINVAL, "dims need %d B of LDS (> %d)", lmax * 4, LDS_MAX);
    }
    return 0;
}

// F2 > 16: o-chunked streaming passes and whole-trial block-2 passes (eegnet_wide.hip)
static int make_geo_wide(Geo* g, bool launch) {
    const int cus = device_cus();
    g->NOC = (g->F2 + 15) / 16;
    g->CPC = (g->C + g->NOC - 1) / g->NOC;
    g->F2P = g->F2 <= 32 ? 32 : 64;
    g->RB = rb_stride(g->T1);
    // streaming grid: one 1024-thread workgroup per CU, NOC per trial range; a multiple of 8 * NOC
    // when it can be (the chunk workgroups of a range then share an XCD)
    int G = std::min(g->B * g->NOC, cus);
    G = std::max(g->NOC, G / g->NOC * g->NOC);
    if (G >= 8 * g->NOC) G = G / (8 * g->NOC) * (8 * g->NOC);
    g->gridS = G;
    g->gridA = g->gridE = G;
    g->grid = std::min(g->B, cus);                      // block-2 passes and the eval forward
    // partial rows wider than this reduce in k_coltail (column-parallel) instead of in-kernel
    g->splitC = g->nC > SPLIT_COLS; g->splitD = g->nD > SPLIT_COLS; g->splitE = g->nE > SPLIT_COLS;
    const int nf4 = rup(g->NF, 4);
    auto tailw = [](int ncols, int fin) { return 2 * (tail_s_doubles(ncols) + fin); };
    const int awl = KSW * 64;                               // spatial GEMM fragment table
    // after the loop pass A's Gram tiles [NWW][16][16 NWT] reuse the slice / s rows when they fit
    const int cgw = NWW * 256 * ((15 + g->K1 - 1) / 16 + 1);
    // the cfg5 shape (k_wpass_a's SPEC instantiation) double-buffers the slice and the s rows
    const bool w5 = g->C == 64 && g->T == 512 && g->F1 == 16 && g->D == 4 && g->K1 == 32;
    const int baseA = (w5 ? 2 : 1) * (g->CPC + 16) * g->RS + NWW * (g->K1 + 1) + 2 * NWW + awl;
    g->ldsWA = std::max(baseA + ((g->CPC + 16) * g->RS >= cgw ? 0 : cgw),
                        tailw(g->nA, std::max(NTH, fin1_scratch_doubles(g->K1, g->F1, g->F2, g->C))));
    g->ldsWB = 0;                                           // k_wpass_b: registers only (v plane)
    const int b2 = 2 * g->F2P * g->RB + g->F2P * K2 + g->F2P * (g->F2P + 1);   // D2, Q, w2, W3 tables
    b2_lds(g, NWB2);
    g->gridB2 = g->grid;
    // the cfg5 (SPEC) k_wpass_b2 keeps its W3 fragments in registers instead of an LDS table, and it and
    // k_wpass_c stay within 128 VGPRs: two 8-wave workgroups per CU, two trials each at B = 1024, so one
    // workgroup's barriers overlap the other's work
    g->gridW2 = w5 ? std::min(g->B, 2 * cus) : g->grid;
    if (w5) g->ldsWB2 = std::max(g->ldsWB2 - g->F2P * (g->F2P + 1), tailw(g->nB, 0));
    // s rows, dy / e rows x 2 (alternate trials), dp2 rows, coefficient table
    g->ldsWE = std::max(std::max(3 * 16 * g->RS + rup(16 * g->T1, 4) + 8 * 16 + awl, NWW * 256 + 32 + NWW * 256 * ((15 + g->K1 - 1) / 16 + 1)),
                        tailw(g->nE, fin5_scratch_doubles(g->K1, g->F1, g->o_g2)));
    g->ldsWI = 16 * g->RS + b2 + nf4 + 4 * g->F2P + g->NOC * awl;
    (void)nf4;
    if (!launch) return 0;
    if (g->C > 4 * KSW) return fail(EEGNET_EINVAL, "C = %d > %d", g->C, 4 * KSW);
    if (g->T1 > 16 * NTTW * (NWB2 / 4)) return fail(EEGNET_EINVAL, "T/4 = %d > %d", g->T1, 16 * NTTW * (NWB2 / 4));
    if (g->NF > MAXNFW * NTB2) return fail(EEGNET_EINVAL, "F2*(T/32) = %d > %d", g->NF, MAXNFW * NTB2);
    if ((double)g->B * g->F2 * g->T1 >= 4294967296.0)
        return fail(EEGNET_EINVAL, "B*F2*(T/4) must stay below 2^32 (dropout / mask indices)");
    const int lmax = std::max(std::max(std::max(g->ldsWA, g->ldsWB), std::max(g->ldsWB2, g->ldsWC)),
                              std::max(std::max(g->ldsWD, g->ldsWE), g->ldsWI));
    if (lmax * 4 > LDS_MAX) return fail(EEGNET_EINVAL, "dims need %d B of LDS (> %d)", lmax * 4, LDS_MAX);
    return 0;
}

static WsLayout make_layout(const Geo& g) {
    WsLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = rupz(o + bytes, 256); return r; };
    L.cnt = take(CNT_BYTES);          // ticket words first: the per-call memset covers [0, CNT_BYTES)
    L.partA = take((size_t)std::max(g.gridS, g.gridA) * g.nA * 4);
    L.partB = take((size_t)std::max(std::max(g.gridS, g.grid), g.gridW2) * g.nB * 4);
    L.partC = take((size_t)std::max(std::max(g.grid, g.gridB2), g.gridW2) * g.nC * 4);
    L.partD = take((size_t)std::max(std::max(g.grid, g.gridB2), g.gridS) * g.nD * 4);   // (k_pass_dr: gridS)
    L.partE = take((size_t)std::max(g.gridS, g.gridE) * g.nE * 4);
    const int nmax = std::max(std::max(std::max(g.nA, g.nB), std::max(g.nC, g.nD)), g.nE);
    L.sums = take((size_t)nmax * 8 * NGRPMAX);
    L.stats = take((size_t)(g.F1 * g.K1 + g.K1) * 8);   // fin1 -> fin5: G w1 per filter, window sums S1
    L.coef = take((size_t)CF_COUNT * CSTR * 4);
    const size_t per = (size_t)g.B * g.F2 * g.T1 * 4;
    L.d2 = take(per); L.E1 = take(per); L.E2 = take(per); L.dp2 = take(per);
    L.dl = take((size_t)g.B * NCLS * 4);
    // pass A's s [B][F2][T] and v [B][F2][8 ceil(T/8)] planes, read back by passes B and E
    L.s = take((size_t)g.B * g.F2 * s_pitch(g.T) * 4);
    L.v = take((size_t)g.B * g.F2 * ((g.T + 7) / 8 * 8) * 4);
    // F2 <= 16: pass B's block-2 depthwise output q and pointwise output r [B][F2][T/4], read by passes
    // C (r) and D (q, r) instead of recomputing them from d2
    L.q3 = take(per);
    L.r3 = take(per);
    L.total = o;
    return L;
}

static uint64_t mix_key(uint64_t seed, uint64_t offset) {
    uint64_t z = seed * 0xD1B54A32D192ED03ull + offset * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// dropout keys of one call: (seed, offset) -> 64-bit key -> two per-layer 32-bit keys, threshold
static void set_key(Geo* g, uint64_t seed, uint64_t offset) {
    g->key = mix_key(seed, offset);
    g->key0 = (unsigned)g->key;
    g->key1 = (unsigned)(g->key >> 32) ^ 0x5BD1E995u;
    g->pthr = (unsigned)std::min(16777216.0, std::max(0.0, (double)g->p * 16777216.0));
}

// ---- optional per-kernel device timing (bench / roofline), off by default ----
enum KernelId { KID_A = 0, KID_B, KID_C, KID_D, KID_E, KID_ADAM, KID_INFER, KID_MEMSET, KID_INFER_BF16,
                KID_WA, KID_WB, KID_WB2, KID_WC, KID_WD, KID_WE, KID_WINFER, KID_CTAIL, KID_XSTATS, KID_COUNT };
static const char* kKernelNames[KID_COUNT] = {"k_pass_a", "k_pass_b", "k_pass_c", "k_pass_d", "k_pass_e",
                                              "k_adam", "k_infer", "memset_tickets", "k_infer_bf16",
                                              "k_wpass_a", "k_wpass_b", "k_wpass_b2", "k_wpass_c", "k_wpass_d",
                                              "k_wpass_e", "k_winfer", "k_coltail", "k_xstats"};
#ifndef EEGNET_PROF_EVENT_FLAGS
#define EEGNET_PROF_EVENT_FLAGS hipEventDisableSystemFence
#endif
struct ProfRec { int kid; hipEvent_t a, b; };
struct ProfState { unsigned mask = 0; std::vector<ProfRec> recs; std::vector<hipEvent_t> pool; };
static thread_local ProfState g_prof;

static hipEvent_t prof_event() {
    if (!g_prof.pool.empty()) { hipEvent_t e = g_prof.pool.back(); g_prof.pool.pop_back(); return e; }
    // timing-only markers: without the system-scope release fence a default event record carries
    // (an L2 writeback + invalidate around the bracketed kernel, ~4 % of a cfg2 step with k_pass_e
    // bracketed every step: profiles/r6zb_event_fence.txt); the times are read after a full device sync
    hipEvent_t e;
    hipEventCreateWithFlags(&e, EEGNET_PROF_EVENT_FLAGS);
    return e;
}
struct ProfScope {
    int kid; hipStream_t s; hipEvent_t a = nullptr;
    ProfScope(int k, hipStream_t st) : kid(k), s(st) {
        if ((g_prof.mask >> k) & 1u) { a = prof_event(); hipEventRecord(a, s); }
    }
    ~ProfScope() {
        if (a) { hipEvent_t b = prof_event(); hipEventRecord(b, s); g_prof.recs.push_back({kid, a, b}); }
    }
};
#define PROF(kid) ProfScope prof_scope_##kid(kid, s)

#define LAUNCH_CHECK(what)                                                            \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) return fail(EEGNET_ELAUNCH, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

static bool g_attr_done = false;

template <int K1, int CC, int TT, int FF>
static void set_attrs_shape() {
    const int lds = LDS_MAX;
    for (const void* f : {(const void*)k_pass_a<K1, CC, TT, FF>, (const void*)k_pass_b<K1, CC, TT, FF>,
                          (const void*)k_pass_c<K1, CC, TT, FF>,
                          (const void*)k_pass_e<K1, CC, TT, FF>, (const void*)k_pass_a<K1, CC, TT, FF, true>,
                          (const void*)k_pass_b<K1, CC, TT, FF, true>, (const void*)k_pass_c<K1, CC, TT, FF, true>,
                          (const void*)k_pass_e<K1, CC, TT, FF, true>,
#if EEGNET_D1
                          (const void*)k_pass_d<K1, CC, TT, FF>, (const void*)k_pass_d<K1, CC, TT, FF, false, false>,
                          (const void*)k_pass_d<K1, CC, TT, FF, true, false>,
#endif
                          (const void*)k_pass_dr<K1, CC, TT, FF>, (const void*)k_pass_dr<K1, CC, TT, FF, false, false>,
                          (const void*)k_pass_dr<K1, CC, TT, FF, true, false>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipFuncSetAttribute((const void*)k_infer<K1, CC, TT, FF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <int K1>
static void set_attrs_wide() {
    for (const void* f : {(const void*)k_wpass_a<K1>, (const void*)k_wpass_b<K1>, (const void*)k_wpass_e<K1>,
                          (const void*)k_winfer<K1>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

static void ensure_attrs() {
    if (g_attr_done) return;
    set_attrs_wide<32>();
    set_attrs_wide<64>();
    for (const void* f : {(const void*)k_wpass_a<32, true>, (const void*)k_wpass_b<32, true>, (const void*)k_wpass_e<32, true>,
                          (const void*)k_winfer<32, true>, (const void*)k_wpass_b2<NTB2, true>,
                          (const void*)k_wpass_c<NTB2, false, true>, (const void*)k_wpass_d<NTB2, false, true>,
                          (const void*)k_coltail<3, true>, (const void*)k_coltail<4, true>, (const void*)k_coltail<5, true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    for (const void* f : {(const void*)k_wpass_b2<NTB2>, (const void*)k_wpass_c<NTB2>, (const void*)k_wpass_d<NTB2>,
                          (const void*)k_wpass_c<256>, (const void*)k_wpass_d<256>,
                          (const void*)k_wpass_c<256, true>, (const void*)k_wpass_d<256, true>,
                          (const void*)k_coltail<3>, (const void*)k_coltail<4>, (const void*)k_coltail<5>,
                          (const void*)k_fin})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    for (const void* f : {(const void*)k_infer_bf16<0>, (const void*)k_infer_bf16<1>, (const void*)k_infer_bf16<2>,
                          (const void*)k_infer_bf16<4>, (const void*)k_infer_bf16<8>, (const void*)k_infer_bf16<16>,
                          (const void*)k_infer_bf16<8, true>, (const void*)k_infer_bf16_cfg5})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    set_attrs_shape<32, 0, 0, 0>();
    set_attrs_shape<64, 0, 0, 0>();
    hipFuncSetAttribute((const void*)k_xstats<32>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    hipFuncSetAttribute((const void*)k_xstats<64>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    set_attrs_shape<32, 22, 256, 16>();
    set_attrs_shape<32, 22, 257, 16>();
    g_attr_done = true;
}

// compile-time shape specialisations (the benchmark and real-data configurations); any other shape
// runs the runtime-shape instantiation of the same kernels
#define EEG_DISPATCH(K1_, g_, LAUNCH)                                                            \
    do {                                                                                         \
        if ((K1_) == 32 && (g_).C == 22 && (g_).T == 256 && (g_).F1 == 8 && (g_).D == 2) { LAUNCH(32, 22, 256, 16); } \
        else if ((K1_) == 32 && (g_).C == 22 && (g_).T == 257 && (g_).F1 == 8 && (g_).D == 2) { LAUNCH(32, 22, 257, 16); } \
        else { LAUNCH(K1_, 0, 0, 0); }                                                           \
    } while (0)

// the finalize arguments of one pass (ticket words `tk`); Adam is attached to pass E by the caller
static FinArgs fin_args(const WsLayout& L, char* ws, int tk, float* bn, float* grads, float* loss,
                        int update_running, int ce, int64_t* nbt = nullptr) {
    FinArgs f;
    memset(&f, 0, sizeof(f));
    f.part2 = (double*)(ws + L.sums);
    f.cnt = (unsigned*)(ws + L.cnt) + tk * NCNT;
    f.stats = (double*)(ws + L.stats);
    f.coef = (float*)(ws + L.coef);
    f.bn = bn; f.grads = grads; f.loss = loss;
    f.update_running = update_running; f.ce = ce;
    f.nbt = nbt;
    f.tpass = tk;
    return f;
}


// the run-time geometry has the compile-time cfg5 shape (eegnet_common.h EEG_SHAPE_W5): launch the
// SPEC instantiations of the wide kernels
static bool same_shape_w5(const Geo& g) {
#define EEG_EQ_(f, v) && g.f == v
    return true EEG_SHAPE_W5(EEG_EQ_);
#undef EEG_EQ_
}
// one wide-kernel launch, SPEC (cfg5 shape, compile-time geometry) or generic
#define WLAUNCH(sp, KG, KS, grid_, blk_, lds_, ...)                                               \
    do {                                                                                          \
        if (sp) hipLaunchKernelGGL(KS, grid_, blk_, lds_, __VA_ARGS__);                           \
        else hipLaunchKernelGGL(KG, grid_, blk_, lds_, __VA_ARGS__);                              \
    } while (0)

// F2 > 16: passes A, B (no reduction), B2 (BN3 statistics)
template <int K1>
static int run_forward_wide(const Geo& g, const WsLayout& L, char* ws, const float* params, float* bn,
                            const float* x, const uint8_t* m2, int update_running, int64_t* nbt, hipStream_t s) {
    const FinArgs fa = fin_args(L, ws, TK_A, bn, nullptr, nullptr, update_running, 0);
    const FinArgs fb = fin_args(L, ws, TK_B, bn, nullptr, nullptr, update_running, 0, nbt);
    const bool sp = K1 == 32 && same_shape_w5(g);
    { PROF(KID_WA); WLAUNCH(sp, (k_wpass_a<K1>), (k_wpass_a<K1, K1 == 32>), dim3(g.gridS), dim3(NTW), g.ldsWA * 4, s, g,
                            params, x, (float*)(ws + L.s), (float*)(ws + L.v), (float*)(ws + L.partA), fa); }
    LAUNCH_CHECK("k_wpass_a");
    // k_wpass_b keeps nothing in LDS and needs 38 VGPRs at cfg5: two 16-wave workgroups per CU (elementwise,
    // so the grid does not touch the numerics)
    { PROF(KID_WB); WLAUNCH(sp, (k_wpass_b<K1>), (k_wpass_b<K1, K1 == 32>), dim3(sp ? std::min(2 * g.gridS, g.B * g.NOC) : g.gridS), dim3(NTW), g.ldsWB * 4, s, g,
                            params, (const float*)(ws + L.coef), (const float*)(ws + L.v), m2, (float*)(ws + L.d2),
                            (float*)(ws + L.E1), (float*)(ws + L.E2)); } LAUNCH_CHECK("k_wpass_b");
    { PROF(KID_WB2); WLAUNCH(sp, k_wpass_b2<NTB2>, (k_wpass_b2<NTB2, true>), dim3(g.gridW2), dim3(NTB2), g.ldsWB2 * 4, s,
                             g, params, (const float*)(ws + L.d2), (float*)(ws + L.q3), (float*)(ws + L.r3),
                             (float*)(ws + L.partB), fb); } LAUNCH_CHECK("k_wpass_b2");
    return 0;
}

template <int K1>
static int run_backward_wide(const Geo& g, const WsLayout& L, char* ws, float* params, const float* x,
                             const uint8_t* m2, const uint8_t* m3, const float* dlogits, const int64_t* labels,
                             float* logits, float* grads, float* loss, int c_mode, const FinArgs* adam,
                             hipStream_t s) {
    const float* coef = (const float*)(ws + L.coef);
    const float* dl = dlogits ? dlogits : (const float*)(ws + L.dl);
    const FinArgs fc = fin_args(L, ws, TK_C, nullptr, grads, loss, 0, (c_mode & PC_CE) ? 1 : 0);
    const FinArgs fd = fin_args(L, ws, TK_D, nullptr, grads, nullptr, 0, 0);
    FinArgs fe = fin_args(L, ws, TK_E, nullptr, grads, nullptr, 0, 0);
    if (adam) {
        fe.params = params; fe.adam_m = adam->adam_m; fe.adam_v = adam->adam_v; fe.step = adam->step;
        fe.lr = adam->lr; fe.b1 = adam->b1; fe.b2 = adam->b2; fe.eps = adam->eps;
    }
    const bool sp = K1 == 32 && same_shape_w5(g);
    // the column-parallel reduction + finalize of a split pass (k_coltail, eegnet_finalize.hip)
    auto coltail = [&](int fin, const float* part, int nrows, int ncols, const FinArgs& fa, int scr) {
        const int nb = (ncols + 63) / 64;
        const size_t lds = 8 * (size_t)std::max(2 + (NTCT / 64) * 64, tail_s_doubles(ncols) + scr);
        PROF(KID_CTAIL);
        if (fin == 3) WLAUNCH(sp, k_coltail<3>, (k_coltail<3, true>), dim3(nb), dim3(NTCT), lds, s, g, (const float*)params, part, nrows, ncols, fa);
        else if (fin == 4) WLAUNCH(sp, k_coltail<4>, (k_coltail<4, true>), dim3(nb), dim3(NTCT), lds, s, g, (const float*)params, part, nrows, ncols, fa);
        else WLAUNCH(sp, k_coltail<5>, (k_coltail<5, true>), dim3(nb), dim3(NTCT), lds, s, g, (const float*)params, part, nrows, ncols, fa);
    };
    { PROF(KID_WC); WLAUNCH(sp, k_wpass_c<NTB2>, (k_wpass_c<NTB2, false, true>), dim3(g.gridW2), dim3(NTB2), g.ldsWC * 4, s,
                            g, params, coef, (const float*)(ws + L.r3), m3, dlogits, labels, logits, (float*)(ws + L.dl),
                            (float*)(ws + L.partC), c_mode, fc, FoldCall{}); } LAUNCH_CHECK("k_wpass_c(bwd)");
    if (g.splitC) { coltail(3, (const float*)(ws + L.partC), g.gridW2, g.nC, fc, 0); LAUNCH_CHECK("k_coltail(C)"); }
    { PROF(KID_WD); WLAUNCH(sp, k_wpass_d<NTB2>, (k_wpass_d<NTB2, false, true>), dim3(g.grid), dim3(NTB2), g.ldsWD * 4, s,
                            g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), (const float*)(ws + L.E2),
                            (const float*)(ws + L.q3), (const float*)(ws + L.r3), m2, m3, dl,
                            (float*)(ws + L.dp2), (float*)(ws + L.partD), fd, FoldCall{}); }
    LAUNCH_CHECK("k_wpass_d");
    if (g.splitD) { coltail(4, (const float*)(ws + L.partD), g.grid, g.nD, fd, 0); LAUNCH_CHECK("k_coltail(D)"); }
    { PROF(KID_WE); WLAUNCH(sp, (k_wpass_e<K1>), (k_wpass_e<K1, K1 == 32>), dim3(g.gridS), dim3(NTW), g.ldsWE * 4, s, g,
                            (const float*)params, coef, x, (const float*)(ws + L.s), (const float*)(ws + L.v),
                            (const float*)(ws + L.dp2), (float*)(ws + L.partE), fe); } LAUNCH_CHECK("k_wpass_e");
    if (g.splitE) {
        // one partial row per trial range (k_wpass_e's chunk workgroups share it, disjoint columns)
        coltail(5, (const float*)(ws + L.partE), g.gridS / g.NOC, g.nE, fe, fin5_scratch_doubles(g.K1, g.F1, g.o_g2));
        LAUNCH_CHECK("k_coltail(E)");
    }
    return 0;
}

// fc.folds != nullptr: fold-indexed launch over nf folds (grid y); the other pointers are unused
template <int K1>
static int run_forward(const Geo& g, const WsLayout& L, char* ws, const float* params, float* bn,
                       const float* x, const uint8_t* m2, int update_running, int64_t* nbt, hipStream_t s,
                       const FoldCall& fc = FoldCall{}, int nf = 1, int only = -1) {
    if (g.wide) return run_forward_wide<K1>(g, L, ws, params, bn, x, m2, update_running, nbt, s);
    const FinArgs fa = fin_args(L, ws, TK_A, bn, nullptr, nullptr, update_running, 0);
    const FinArgs fb = fin_args(L, ws, TK_B, bn, nullptr, nullptr, update_running, 0, nbt);
#define LAUNCH_A(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_a<K, CC, TT, FF, true>), dim3(g.gridA, nf), dim3(NTB), g.ldsA * 4, s, \
                                                   g, params, x, (float*)(ws + L.s), (float*)(ws + L.v), (float*)(ws + L.partA), fa, fc); \
    else hipLaunchKernelGGL((k_pass_a<K, CC, TT, FF>), dim3(g.gridA, nf), dim3(NTB), g.ldsA * 4, s, \
                                                   g, params, x, (float*)(ws + L.s), (float*)(ws + L.v), (float*)(ws + L.partA), fa, fc)
    if (only < 0 || only == 0) { { PROF(KID_A); EEG_DISPATCH(K1, g, LAUNCH_A);
    } LAUNCH_CHECK("k_pass_a"); }
#define LAUNCH_B(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_b<K, CC, TT, FF, true>), dim3(g.gridS, nf), dim3(NTB), g.ldsB * 4, s, \
                       g, params, (const float*)(ws + L.coef), (const float*)(ws + L.v), m2, (float*)(ws + L.d2), \
                       (float*)(ws + L.E1), (float*)(ws + L.E2), (float*)(ws + L.q3), (float*)(ws + L.r3), \
                       (float*)(ws + L.partB), fb, fc); \
    else hipLaunchKernelGGL((k_pass_b<K, CC, TT, FF>), dim3(g.gridS, nf), dim3(NTB), g.ldsB * 4, s, \
                       g, params, (const float*)(ws + L.coef), (const float*)(ws + L.v), m2, (float*)(ws + L.d2), \
                       (float*)(ws + L.E1), (float*)(ws + L.E2), (float*)(ws + L.q3), (float*)(ws + L.r3), \
                       (float*)(ws + L.partB), fb, fc)
    if (only < 0 || only == 1) { { PROF(KID_B); EEG_DISPATCH(K1, g, LAUNCH_B);
    } LAUNCH_CHECK("k_pass_b"); }
    return 0;
}

// adam: nullptr = gradients only
template <int K1>
static int run_backward(const Geo& g, const WsLayout& L, char* ws, float* params,
                        const float* x, const uint8_t* m2, const uint8_t* m3, const float* dlogits,
                        const int64_t* labels, float* logits, float* grads, float* loss, int c_mode,
                        const FinArgs* adam, hipStream_t s, const FoldCall& fc = FoldCall{}, int nf = 1,
                        int only = -1) {
    if (g.wide)
        return run_backward_wide<K1>(g, L, ws, params, x, m2, m3, dlogits, labels, logits, grads, loss, c_mode,
                                     adam, s);
    const float* coef = (const float*)(ws + L.coef);
    const float* dl = dlogits ? dlogits : (const float*)(ws + L.dl);
    const FinArgs fcC = fin_args(L, ws, TK_C, nullptr, grads, loss, 0, (c_mode & PC_CE) ? 1 : 0);
    const FinArgs fd = fin_args(L, ws, TK_D, nullptr, grads, nullptr, 0, 0);
    FinArgs fe = fin_args(L, ws, TK_E, nullptr, grads, nullptr, 0, 0);
    if (adam) {
        fe.params = params; fe.adam_m = adam->adam_m; fe.adam_v = adam->adam_v; fe.step = adam->step;
        fe.lr = adam->lr; fe.b1 = adam->b1; fe.b2 = adam->b2; fe.eps = adam->eps;
    }
#define LAUNCH_CB(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_c<K, CC, TT, FF, true>), dim3(g.grid, nf), dim3(64 * g.nwC), g.ldsC * 4, s, \
                       g, params, coef, (const float*)(ws + L.r3), m3, dlogits, labels, logits, \
                       (float*)(ws + L.dl), (float*)(ws + L.partC), c_mode, fcC, fc); \
    else hipLaunchKernelGGL((k_pass_c<K, CC, TT, FF>), dim3(g.grid, nf), dim3(64 * g.nwC), g.ldsC * 4, s, \
                       g, params, coef, (const float*)(ws + L.r3), m3, dlogits, labels, logits, \
                       (float*)(ws + L.dl), (float*)(ws + L.partC), c_mode, fcC, fc)
    if (use_b2_narrow(g)) {
        if (only >= 0) return fail(EEGNET_EINVAL, "staged steps do not support EEGNET_B2=1");
        { PROF(KID_C);
          if (fc.folds) hipLaunchKernelGGL((k_wpass_c<256, true>), dim3(g.gridB2, nf), dim3(256), g.ldsWC * 4, s, g,
                                           params, coef, (const float*)(ws + L.r3), m3, dlogits, labels, logits,
                                           (float*)(ws + L.dl), (float*)(ws + L.partC), c_mode, fcC, fc);
          else hipLaunchKernelGGL((k_wpass_c<256>), dim3(g.gridB2), dim3(256), g.ldsWC * 4, s, g, params, coef,
                                  (const float*)(ws + L.r3), m3, dlogits, labels, logits, (float*)(ws + L.dl),
                                  (float*)(ws + L.partC), c_mode, fcC, fc);
        } LAUNCH_CHECK("k_wpass_c<256>");
        { PROF(KID_D);
          if (fc.folds) hipLaunchKernelGGL((k_wpass_d<256, true>), dim3(g.gridB2, nf), dim3(256), g.ldsWD * 4, s, g,
                                           params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1),
                                           (const float*)(ws + L.E2), (const float*)(ws + L.q3),
                                           (const float*)(ws + L.r3), m2, m3, dl, (float*)(ws + L.dp2),
                                           (float*)(ws + L.partD), fd, fc);
          else hipLaunchKernelGGL((k_wpass_d<256>), dim3(g.gridB2), dim3(256), g.ldsWD * 4, s, g, params, coef,
                                  (const float*)(ws + L.d2), (const float*)(ws + L.E1), (const float*)(ws + L.E2),
                                  (const float*)(ws + L.q3), (const float*)(ws + L.r3), m2, m3, dl,
                                  (float*)(ws + L.dp2), (float*)(ws + L.partD), fd, fc);
        } LAUNCH_CHECK("k_wpass_d<256>");
    } else {
    if (only < 0 || only == 2) { { PROF(KID_C); EEG_DISPATCH(K1, g, LAUNCH_CB);
    } LAUNCH_CHECK("k_pass_c(bwd)"); }
#define LAUNCH_DR(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_dr<K, CC, TT, FF, true, false>), dim3(g.gridS, nf), dim3(NTB), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc); \
    else if (m2 || m3) hipLaunchKernelGGL((k_pass_dr<K, CC, TT, FF>), dim3(g.gridS, nf), dim3(NTB), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc); \
    else hipLaunchKernelGGL((k_pass_dr<K, CC, TT, FF, false, false>), dim3(g.gridS, nf), dim3(NTB), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc)
#define LAUNCH_D(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_d<K, CC, TT, FF, true, false>), dim3(g.grid, nf), dim3(64 * g.nwD), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc); \
    else if (m2 || m3) hipLaunchKernelGGL((k_pass_d<K, CC, TT, FF>), dim3(g.grid, nf), dim3(64 * g.nwD), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc); \
    else hipLaunchKernelGGL((k_pass_d<K, CC, TT, FF, false, false>), dim3(g.grid, nf), dim3(64 * g.nwD), g.ldsD * 4, s, \
                       g, params, coef, (const float*)(ws + L.d2), (const float*)(ws + L.E1), \
                       (const float*)(ws + L.E2), (const float*)(ws + L.q3), (const float*)(ws + L.r3), \
                       m2, m3, dl, (float*)(ws + L.dp2), \
                       (float*)(ws + L.partD), fd, fc)
#if EEGNET_D1
#define LAUNCH_PASS_D LAUNCH_D
#else
#define LAUNCH_PASS_D LAUNCH_DR
#endif
    if (only < 0 || only == 3) { { PROF(KID_D); EEG_DISPATCH(K1, g, LAUNCH_PASS_D);
    } LAUNCH_CHECK("k_pass_d"); }
    }
#define LAUNCH_E(K, CC, TT, FF) if (fc.folds) hipLaunchKernelGGL((k_pass_e<K, CC, TT, FF, true>), dim3(g.gridE, nf), dim3(NTB), g.ldsE * 4, s, \
                       g, (const float*)params, coef, x, (const float*)(ws + L.s), (const float*)(ws + L.v), \
                       (const float*)(ws + L.dp2), (float*)(ws + L.partE), fe, fc); \
    else hipLaunchKernelGGL((k_pass_e<K, CC, TT, FF>), dim3(g.gridE, nf), dim3(NTB), g.ldsE * 4, s, \
                       g, (const float*)params, coef, x, (const float*)(ws + L.s), (const float*)(ws + L.v), \
                       (const float*)(ws + L.dp2), (float*)(ws + L.partE), fe, fc)
    if (only < 0 || only == 4) { { PROF(KID_E); EEG_DISPATCH(K1, g, LAUNCH_E);
    } LAUNCH_CHECK("k_pass_e"); }
    return 0;
}

#ifndef EEGNET_BF16_V1
#define EEGNET_BF16_V1 0
#endif
// geometry of the bf16 eval kernel (eegnet_infer_bf16.hip)
static float* g_bf16_dbg = nullptr;     // eegnet_debug_bf16 (debug builds only)

static int make_geo_bf16(const eegnet_dims* d, GeoI* g) {
    Geo q;
    if (int r = make_geo(d, &q, false)) return r;
    memset(g, 0, sizeof(*g));
    g->B = q.B; g->C = q.C; g->T = q.T; g->F1 = q.F1; g->D = q.D; g->F2 = q.F2; g->K1 = q.K1; g->P = q.P;
    g->eps = q.eps;
    g->o_w1 = q.o_w1; g->o_g1 = q.o_g1; g->o_b1 = q.o_b1; g->o_ws = q.o_ws; g->o_g2 = q.o_g2;
    g->o_b2 = q.o_b2; g->o_w2 = q.o_w2; g->o_W3 = q.o_W3; g->o_g3 = q.o_g3; g->o_b3 = q.o_b3;
    g->o_Wfc = q.o_Wfc; g->o_bfc = q.o_bfc;
    g->CP = rup(g->C, 32); g->KC = g->CP / 32;
    g->F2P = g->F2 <= 16 ? 16 : g->F2 <= 32 ? 32 : 64;
    g->NOT = g->F2P / 16;
    g->F2K = std::max(32, g->F2P); g->KCW = g->F2K / 32;
    g->TX = rup(g->T, 128);
    g->NT = (g->T + 15) / 16; g->NBLK = (g->NT + 15) / 16;
    g->LPs = g->P + 1;
    g->KSF = (g->K1 + 16 + 31) / 32;
    // s rows: FIR windows read up to element 256*NBLK + 32*KSF - 16; row stride = 4 mod 8 dwords so the
    // 16 rows of one spatial-tile store land on distinct bank quads
    g->SXs = 256 * g->NBLK + 32 * g->KSF - 8;
    g->T1 = g->T / 4; g->T2 = g->T1 / 8; g->NF = g->F2 * g->T2;
    const int nq = (g->T1 + 3) / 4;
    g->RA = 4 * nq + 16;
    g->NT1 = (8 * g->T2 + 15) / 16;
    g->TZ = rup(std::max(4 * nq, 16 * g->NT1), 128);
    if (g->T % 8 == 0) {
        const int units = g->CP * g->TX / 8;
        int u = (units + NTI - 1) / NTI, p = 1;
        while (p < u) p *= 2;
        g->PFU = p;
    } else {
        g->PFU = 0;
    }
    if (g->PFU > 16) return fail(EEGNET_EINVAL, "bf16 eval: C*T too large for one trial in registers");
    const int r1 = std::max(g->CP * g->TX * 2, rup(g->F2P * g->RA * 4, 16) + g->F2K * g->TZ * 2);
    g->offZ = rup(g->F2P * g->RA * 4, 16);
    g->offS = rup(r1, 16);
    g->offW1 = rup(g->offS + g->F2P * g->SXs * 2, 16);
    g->offW2 = rup(g->offW1 + g->F1 * g->K1 * 4, 16);
    g->offCo = rup(g->offW2 + g->F2P * K2 * 4, 16);
    g->offL = rup(g->offCo + 4 * g->F2P * 4, 16);
    g->lds = g->offL + NWI * NCLS * 4;
    // classifier weights staged in LDS when they fit (cfg5: 16 KB), else read from global
    const int offF = rup(g->lds, 16);
    if (offF + NCLS * g->NF * 4 <= LDS_MAX) {
        g->offF = offF;
        g->lds = offF + NCLS * g->NF * 4;
    }
    g->dbg = g_bf16_dbg;
    if (g->lds > LDS_MAX)
        return fail(EEGNET_EINVAL, "bf16 eval: dims need %d B of LDS (> %d): C=%d T=%d F2=%d", g->lds, LDS_MAX,
                    g->C, g->T, g->F2);
    return 0;
}

// every shape-derived field equal (B, eps and the debug pointer are runtime in every instantiation)
static bool same_geo_bf16(GeoI a, GeoI b) {
    a.B = b.B = 0;
    a.eps = b.eps = 0.f;
    a.dbg = b.dbg = nullptr;
    return memcmp(&a, &b, sizeof(GeoI)) == 0;
}

static int check_ptrs(const void* a, const char* na, const void* b = (const void*)1, const char* nb = "") {
    if (!a) return fail(EEGNET_EINVAL, "%s is NULL", na);
    if (!b) return fail(EEGNET_EINVAL, "%s is NULL", nb);
    return 0;
}

extern "C" {

int eegnet_param_count(const eegnet_dims* dims, int64_t* out) {
    Geo g;
    if (int r = make_geo(dims, &g, false)) return r;
    if (!out) return fail(EEGNET_EINVAL, "out is NULL");
    *out = g.nparam;
    return 0;
}

int eegnet_x_pitch(const eegnet_dims* dims) {
    if (!dims) return fail(EEGNET_EINVAL, "dims is NULL");
    return x_pitch_shape(*dims) && (dims->T & 3) ? (dims->T + 3) & ~3 : dims->T;
}

int eegnet_wide_spec(const eegnet_dims* dims) {
    Geo g;
    memset(&g, 0, sizeof(g));
    if (int r = make_geo(dims, &g, false)) return r;
    if (!g.wide || g.K1 != 32) return 0;
    if (same_shape_w5(g)) return 1;
    std::string msg = "geometry differs from EEG_SHAPE_W5:";
    char b[96];
#define EEG_DIFF_(f, v) if (g.f != v) { snprintf(b, sizeof(b), " %s = %d (compiled %d)", #f, (int)g.f, v); msg += b; }
    EEG_SHAPE_W5(EEG_DIFF_)
#undef EEG_DIFF_
    g_err = msg;
    return 0;
}

int eegnet_workspace_bytes(const eegnet_dims* dims, size_t* out) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (!out) return fail(EEGNET_EINVAL, "out is NULL");
    *out = make_layout(g).total;
    return 0;
}

int eegnet_forward_train(const eegnet_dims* dims, const float* params, float* bn_buffers,
                         const float* x, const uint8_t* mask2, const uint8_t* mask3,
                         uint64_t seed, uint64_t offset, float* logits, void* ws, void* stream,
                         int64_t* num_batches_tracked) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", logits, "logits")) return r;
    if (int r = check_ptrs(ws, "ws")) return r;
    g.drop = g.p > 0.f ? 1 : 0;
    set_key(&g, seed, offset);
    ensure_attrs();
    const WsLayout L = make_layout(g);
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    int r = g.K1 == 32 ? run_forward<32>(g, L, w, params, bn_buffers, x, mask2, 1, num_batches_tracked, s)
                       : run_forward<64>(g, L, w, params, bn_buffers, x, mask2, 1, num_batches_tracked, s);
    if (r) return r;
    FinArgs none;
    memset(&none, 0, sizeof(none));
    if (g.wide) {
        const bool sp = g.K1 == 32 && same_shape_w5(g);
        { PROF(KID_WC); WLAUNCH(sp, k_wpass_c<NTB2>, (k_wpass_c<NTB2, false, true>), dim3(g.gridW2), dim3(NTB2),
                                g.ldsWC * 4, s, g, params, (const float*)(w + L.coef), (const float*)(w + L.r3), mask3,
                                (const float*)nullptr, (const int64_t*)nullptr, logits, (float*)nullptr,
                                (float*)nullptr, (int)PC_LOGITS, none, FoldCall{}); }
        LAUNCH_CHECK("k_wpass_c(fwd)");
        return 0;
    }
#define LAUNCH_CF(K, CC, TT, FF) hipLaunchKernelGGL((k_pass_c<K, CC, TT, FF>), dim3(g.grid), dim3(64 * g.nwC), g.ldsC * 4, s, \
                       g, params, (const float*)(w + L.coef), (const float*)(w + L.r3), mask3, (const float*)nullptr, \
                       (const int64_t*)nullptr, logits, (float*)nullptr, (float*)nullptr, (int)PC_LOGITS, none, \
                       FoldCall{})
    { PROF(KID_C);
      if (g.K1 == 32) EEG_DISPATCH(32, g, LAUNCH_CF); else EEG_DISPATCH(64, g, LAUNCH_CF);
    } LAUNCH_CHECK("k_pass_c(fwd)");
    return 0;
}

int eegnet_backward(const eegnet_dims* dims, const float* params, const float* x,
                    const float* dlogits, const int64_t* labels, const uint8_t* mask2,
                    const uint8_t* mask3, uint64_t seed, uint64_t offset, float* grads, float* loss,
                    void* ws, void* stream, int flags) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    g.noclamp = (flags & EEGNET_NO_CLAMP) ? 1 : 0;
    if (int r = check_ptrs(params, "params", x, "x")) return r;
    if (int r = check_ptrs(grads, "grads", ws, "ws")) return r;
    if (!dlogits && !labels) return fail(EEGNET_EINVAL, "need dlogits or labels");
    g.drop = g.p > 0.f ? 1 : 0;
    set_key(&g, seed, offset);
    ensure_attrs();
    const WsLayout L = make_layout(g);
    const int mode = PC_BWD | (dlogits ? 0 : PC_CE);
    hipStream_t s = (hipStream_t)stream;
    float* p = const_cast<float*>(params);        // written only by a fused Adam, which this call has not
    return g.K1 == 32
        ? run_backward<32>(g, L, (char*)ws, p, x, mask2, mask3, dlogits, labels, nullptr, grads, loss, mode, nullptr, s)
        : run_backward<64>(g, L, (char*)ws, p, x, mask2, mask3, dlogits, labels, nullptr, grads, loss, mode, nullptr, s);
}

int eegnet_forward_eval(const eegnet_dims* dims, const float* params, const float* bn_buffers,
                        const float* x, float* logits, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (g.XP != g.T) return fail(EEGNET_EINVAL, "the eval forward takes x as [B][C][T] (x_pitch 0 or T)");
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", logits, "logits")) return r;
    ensure_attrs();
    hipStream_t s = (hipStream_t)stream;
    if (g.wide) {
        PROF(KID_WINFER);
        if (g.K1 == 32) WLAUNCH(same_shape_w5(g), k_winfer<32>, (k_winfer<32, true>), dim3(g.grid), dim3(NTW), g.ldsWI * 4, s,
                                g, params, bn_buffers, x, logits);
        else hipLaunchKernelGGL(k_winfer<64>, dim3(g.grid), dim3(NTW), g.ldsWI * 4, s, g, params, bn_buffers, x, logits);
        LAUNCH_CHECK("k_winfer");
        return 0;
    }
    PROF(KID_INFER);
#define LAUNCH_I(K, CC, TT, FF) hipLaunchKernelGGL((k_infer<K, CC, TT, FF>), dim3(g.grid), dim3(NTH), g.ldsI * 4, s, \
                                                   g, params, bn_buffers, x, logits)
    if (g.K1 == 32) EEG_DISPATCH(32, g, LAUNCH_I); else EEG_DISPATCH(64, g, LAUNCH_I);
    LAUNCH_CHECK("k_infer");
    return 0;
}

int eegnet_forward_eval_bf16(const eegnet_dims* dims, const float* params, const float* bn_buffers,
                             const uint16_t* x, float* logits, void* stream) {
    GeoI g;
    if (int r = make_geo_bf16(dims, &g)) return r;
    if (dims->x_pitch && dims->x_pitch != dims->T)
        return fail(EEGNET_EINVAL, "the eval forward takes x as [B][C][T] (x_pitch 0 or T)");
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", logits, "logits")) return r;
    if (g.PFU > 0 && ((uintptr_t)x & 15))
        return fail(EEGNET_EINVAL, "bf16 eval: x must be 16-byte aligned");
    ensure_attrs();
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(std::min(g.B, device_cus())), blk(NTI);
    PROF(KID_INFER_BF16);
    if (same_geo_bf16(g, kGeoCfg5)) {
        // time-chunked cfg5 kernel, two workgroups per CU (eegnet_infer_bf16c.hip); a -DEEGNET_BF16_V1=1
        // build keeps the whole-trial kernel (A/B measurements)
        if (EEGNET_BF16_V1 == 1) hipLaunchKernelGGL((k_infer_bf16<8, true>), grid, blk, g.lds, s, g, params, bn_buffers, x, logits);
        else hipLaunchKernelGGL(k_infer_bf16_cfg5, dim3(std::min(g.B, 2 * device_cus())), dim3(c5::NT), c5::LDS, s,
                                g, params, bn_buffers, x, logits);
        LAUNCH_CHECK("k_infer_bf16(cfg5)");
        return 0;
    }
    switch (g.PFU) {
        case 0: hipLaunchKernelGGL(k_infer_bf16<0>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
        case 1: hipLaunchKernelGGL(k_infer_bf16<1>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
        case 2: hipLaunchKernelGGL(k_infer_bf16<2>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
        case 4: hipLaunchKernelGGL(k_infer_bf16<4>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
        case 8: hipLaunchKernelGGL(k_infer_bf16<8>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
        default: hipLaunchKernelGGL(k_infer_bf16<16>, grid, blk, g.lds, s, g, params, bn_buffers, x, logits); break;
    }
    LAUNCH_CHECK("k_infer_bf16");
    return 0;
}

int eegnet_adam_step(int64_t n, float* params, const float* grads, float* exp_avg,
                     float* exp_avg_sq, int32_t* step, float lr, float beta1, float beta2,
                     float eps, void* stream) {
    if (n <= 0) return fail(EEGNET_EINVAL, "n must be > 0");
    if (!params || !grads || !exp_avg || !exp_avg_sq || !step) return fail(EEGNET_EINVAL, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    { PROF(KID_ADAM); hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, params, grads,
                       exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps);
    } LAUNCH_CHECK("k_adam");
    hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(64), 0, s, step);
    LAUNCH_CHECK("k_step_inc");
    return 0;
}

int eegnet_train_step(const eegnet_dims* dims, float* params, float* bn_buffers, const float* x,
                      const int64_t* labels, uint64_t seed, uint64_t offset, float* grads,
                      float* adam_state, int32_t* step, float lr, float beta1, float beta2,
                      float eps, float* loss, float* logits, void* ws, void* stream, int flags,
                      int64_t* num_batches_tracked) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", labels, "labels")) return r;
    if (int r = check_ptrs(grads, "grads", ws, "ws")) return r;
    if (adam_state && !step) return fail(EEGNET_EINVAL, "step is NULL");
    if (flags & ~(EEGNET_NO_CLAMP | EEGNET_KEY_FROM_STEP))
        return fail(EEGNET_EINVAL, "unknown flags 0x%x (bit 4, round 5's opt-in persistent step, is retired)",
                    flags & ~(EEGNET_NO_CLAMP | EEGNET_KEY_FROM_STEP));
    g.noclamp = (flags & EEGNET_NO_CLAMP) ? 1 : 0;
    g.drop = g.p > 0.f ? 1 : 0;
    set_key(&g, seed, offset);
    if (flags & EEGNET_KEY_FROM_STEP) {
        if (!step) return fail(EEGNET_EINVAL, "EEGNET_KEY_FROM_STEP needs the device step counter");
        g.keystep = step; g.kseed = seed; g.koff = offset;
    }
    ensure_attrs();
    const WsLayout L = make_layout(g);
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    int r = g.K1 == 32 ? run_forward<32>(g, L, w, params, bn_buffers, x, nullptr, 1, num_batches_tracked, s)
                       : run_forward<64>(g, L, w, params, bn_buffers, x, nullptr, 1, num_batches_tracked, s);
    if (r) return r;
    const int mode = PC_BWD | PC_CE | (logits ? PC_LOGITS : 0);
    // Adam runs in pass E's finalize; adam_state == NULL: gradients only (data-parallel: all-reduce,
    // clamp, then eegnet_adam_step)
    FinArgs adam;
    memset(&adam, 0, sizeof(adam));
    adam.adam_m = adam_state; adam.adam_v = adam_state ? adam_state + g.nparam : nullptr; adam.step = step;
    adam.lr = lr; adam.b1 = beta1; adam.b2 = beta2; adam.eps = eps;
    const FinArgs* ap = adam_state ? &adam : nullptr;
    return g.K1 == 32
        ? run_backward<32>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, logits, grads, loss, mode, ap, s)
        : run_backward<64>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, logits, grads, loss, mode, ap, s);
}

// One stage of a data-parallel train step with synchronised BatchNorm (distributed.py
// DataParallelTrainer(sync_bn=True)): stage 2k launches pass k (A..E) with its finalize deferred --
// the reduction's winner leaves the pass's fp64 sums at eegnet_stage_sums' place in the workspace for
// the host to all-reduce over the ranks --, stage 2k + 1 runs pass k's finalize (k_fin) on the reduced
// sums.  norm_batch: the global batch (BN statistics, the CE mean), so every finalize sees global-batch
// sums and the gradients, running statistics, clamps and Adam come out identical on every rank.
int eegnet_train_stage(const eegnet_dims* dims, int stage, int64_t norm_batch, float* params, float* bn_buffers,
                       const float* x, const int64_t* labels, uint64_t seed, uint64_t offset, float* grads,
                       float* adam_state, int32_t* step, float lr, float beta1, float beta2, float eps,
                       float* loss, void* ws, void* stream, int flags, int64_t* num_batches_tracked) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (g.wide) return fail(EEGNET_EINVAL, "eegnet_train_stage: F1*D = %d > 16 is not supported", g.F2);
    if (stage < 0 || stage >= 2 * TK_COUNT) return fail(EEGNET_EINVAL, "stage must be in [0, %d) (got %d)", 2 * TK_COUNT, stage);
    if (norm_batch < g.B || norm_batch > (1LL << 30))
        return fail(EEGNET_EINVAL, "norm_batch must be in [B, 2^30] (got %lld)", (long long)norm_batch);
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", labels, "labels")) return r;
    if (int r = check_ptrs(grads, "grads", ws, "ws")) return r;
    if (adam_state && !step) return fail(EEGNET_EINVAL, "step is NULL");
    g.Bn = (int)norm_batch;
    g.noclamp = (flags & EEGNET_NO_CLAMP) ? 1 : 0;
    g.drop = g.p > 0.f ? 1 : 0;
    set_key(&g, seed, offset);
    if (flags & EEGNET_KEY_FROM_STEP) {
        if (!step) return fail(EEGNET_EINVAL, "EEGNET_KEY_FROM_STEP needs the device step counter");
        g.keystep = step; g.kseed = seed; g.koff = offset;
    }
    ensure_attrs();
    const WsLayout L = make_layout(g);
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    const int pass = stage >> 1;
    FinArgs adam;
    memset(&adam, 0, sizeof(adam));
    adam.adam_m = adam_state; adam.adam_v = adam_state ? adam_state + g.nparam : nullptr; adam.step = step;
    adam.lr = lr; adam.b1 = beta1; adam.b2 = beta2; adam.eps = eps;
    g.defer = 1;                  // (k_fin: fin5 runs the whole Adam update, adam_early is off)
    if ((stage & 1) == 0) {
        if (pass < 2)
            return g.K1 == 32 ? run_forward<32>(g, L, w, params, bn_buffers, x, nullptr, 1, num_batches_tracked, s, FoldCall{}, 1, pass)
                              : run_forward<64>(g, L, w, params, bn_buffers, x, nullptr, 1, num_batches_tracked, s, FoldCall{}, 1, pass);
        const int mode = PC_BWD | PC_CE;
        return g.K1 == 32
            ? run_backward<32>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, nullptr, grads, loss, mode, nullptr, s, FoldCall{}, 1, pass)
            : run_backward<64>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, nullptr, grads, loss, mode, nullptr, s, FoldCall{}, 1, pass);
    }
    FinArgs fa;
    int ncols, lds;
    switch (pass) {
        case 0: fa = fin_args(L, w, TK_A, bn_buffers, nullptr, nullptr, 1, 0); ncols = g.nA; lds = g.ldsA; break;
        case 1: fa = fin_args(L, w, TK_B, bn_buffers, nullptr, nullptr, 1, 0, num_batches_tracked); ncols = g.nB; lds = g.ldsB; break;
        case 2: fa = fin_args(L, w, TK_C, nullptr, grads, loss, 0, 1); ncols = g.nC; lds = g.ldsC; break;
        case 3: fa = fin_args(L, w, TK_D, nullptr, grads, nullptr, 0, 0); ncols = g.nD; lds = g.ldsD; break;
        default:
            fa = fin_args(L, w, TK_E, nullptr, grads, nullptr, 0, 0); ncols = g.nE; lds = g.ldsE;
            if (adam_state) {
                fa.params = params; fa.adam_m = adam.adam_m; fa.adam_v = adam.adam_v; fa.step = step;
                fa.lr = lr; fa.b1 = beta1; fa.b2 = beta2; fa.eps = eps;
            }
            break;
    }
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(NTB), (size_t)lds * 4, s, g, (const float*)params, fa, pass, ncols);
    LAUNCH_CHECK("k_fin");
    return 0;
}

// where stage 2k leaves pass k's sums in a workspace: byte offset and count of fp64 values
int eegnet_stage_sums(const eegnet_dims* dims, int pass, size_t* offset_bytes, int* count) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (pass < 0 || pass >= TK_COUNT) return fail(EEGNET_EINVAL, "pass must be in [0, %d) (got %d)", TK_COUNT, pass);
    if (!offset_bytes || !count) return fail(EEGNET_EINVAL, "null output pointer");
    const WsLayout L = make_layout(g);
    *offset_bytes = L.sums;
    const int n[TK_COUNT] = {g.nA, g.nB, g.nC, g.nD, g.nE};
    *count = n[pass];
    return 0;
}

}  // extern "C"

// trials per workgroup of the fold-indexed launches: the streaming-grid passes A / B / D (k_pass_dr) /
// E, pass C, the whole-trial block-2 passes (-DEEGNET_B2=1); a -DEEGNET_FOLD_TPW_S / _C / _B2 build
// overrides them (sweeps, tools/r6_tpw.sh).  Chosen over 12, 23, 45 and 90 resident folds of batch 64
// (22 x 257): 4 trials per streaming workgroup; pass C one trial per wave of its 16 (round 6:
// 16 instead of 8 left no wave idle, +3 % at 12 folds and +5-6 % at 45 / 90).
#ifndef EEGNET_FOLD_TPW_S
#define EEGNET_FOLD_TPW_S 4
#endif
#ifndef EEGNET_FOLD_TPW_A
#define EEGNET_FOLD_TPW_A EEGNET_FOLD_TPW_S
#endif
#ifndef EEGNET_FOLD_TPW_E
#define EEGNET_FOLD_TPW_E EEGNET_FOLD_TPW_S
#endif
#ifndef EEGNET_FOLD_TPW_C
#define EEGNET_FOLD_TPW_C 16
#endif
#ifndef EEGNET_FOLD_TPW_B2
#define EEGNET_FOLD_TPW_B2 2
#endif
static void fold_tpw(int* s, int* c, int* b2) {
    *s = EEGNET_FOLD_TPW_S; *c = EEGNET_FOLD_TPW_C; *b2 = EEGNET_FOLD_TPW_B2;
}

extern "C" {

int eegnet_train_step_folds(const eegnet_dims* dims, int nfolds, const eegnet_fold* folds, int64_t row0,
                            int64_t slot, uint64_t offset, float lr, float beta1, float beta2, float eps,
                            void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (g.wide) return fail(EEGNET_EINVAL, "eegnet_train_step_folds: F1*D = %d > 16 is not supported", g.F2);
    if (nfolds < 1 || nfolds > 65535) return fail(EEGNET_EINVAL, "nfolds must be in [1, 65535] (got %d)", nfolds);
    if (!folds) return fail(EEGNET_EINVAL, "folds is NULL");
    if (row0 < 0 || slot < 0) return fail(EEGNET_EINVAL, "row0 / slot must be >= 0");
    g.drop = g.p > 0.f ? 1 : 0;
    set_key(&g, 0, offset);                           // the keep threshold (keys come per fold)
    ensure_attrs();
    const WsLayout L = make_layout(g);
    // the folds share the chip: each workgroup runs several trials of its fold (its prologue and the
    // reduction tail are per workgroup).  The per-fold grid is a function of B alone -- never of
    // nfolds -- so a fold's trial -> workgroup split, and with it every partial sum and every bit of
    // its result, does not depend on how many folds share the launch (fold-batch width, sharding
    // over ranks).  Capped at the non-fold grids the workspace's partial rows are sized for.
    int tpwS, tpwC, tpwB2;
    fold_tpw(&tpwS, &tpwC, &tpwB2);
    g.gridA = std::max(1, std::min(g.gridS, (g.B + EEGNET_FOLD_TPW_A - 1) / EEGNET_FOLD_TPW_A));
    g.gridE = std::max(1, std::min(g.gridS, (g.B + EEGNET_FOLD_TPW_E - 1) / EEGNET_FOLD_TPW_E));
    g.gridS = std::max(1, std::min(g.gridS, (g.B + tpwS - 1) / tpwS));
    g.grid = std::max(1, std::min(g.grid, (g.B + tpwC - 1) / tpwC));
    g.gridB2 = std::max(1, std::min(g.gridB2, (g.B + tpwB2 - 1) / tpwB2));
    FoldCall fc;
    memset(&fc, 0, sizeof(fc));
    fc.folds = folds;
    fc.row0 = row0; fc.slot = slot; fc.koff = offset;
    fc.lr = lr; fc.b1 = beta1; fc.b2 = beta2; fc.eps = eps;
    fc.off = {L.cnt, L.partA, L.partB, L.partC, L.partD, L.partE, L.sums, L.stats, L.coef, L.d2, L.E1, L.E2,
              L.dp2, L.dl, L.s, L.v, L.q3, L.r3};
    hipStream_t s = (hipStream_t)stream;
    FinArgs adam;                                     // non-null marker: pass E's finalize runs Adam
    memset(&adam, 0, sizeof(adam));
    char* w = nullptr;                                // every per-fold pointer comes from `folds`
    int r = g.K1 == 32 ? run_forward<32>(g, L, w, nullptr, nullptr, nullptr, nullptr, 1, nullptr, s, fc, nfolds)
                       : run_forward<64>(g, L, w, nullptr, nullptr, nullptr, nullptr, 1, nullptr, s, fc, nfolds);
    if (r) return r;
    const int mode = PC_BWD | PC_CE;
    return g.K1 == 32
        ? run_backward<32>(g, L, w, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           mode, &adam, s, fc, nfolds)
        : run_backward<64>(g, L, w, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           mode, &adam, s, fc, nfolds);
}

int eegnet_x_stats_width(const eegnet_dims* dims) {
    Geo g;
    if (int r = make_geo(dims, &g, false)) return r;
    if (g.wide) return fail(EEGNET_EINVAL, "eegnet_x_stats: F1*D = %d > 16 is not supported", g.F2);
    return g.K1 + 1 + g.nedge;
}

int eegnet_x_stats(const eegnet_dims* dims, int64_t n, const float* x, float* out, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (g.wide) return fail(EEGNET_EINVAL, "eegnet_x_stats: F1*D = %d > 16 is not supported", g.F2);
    if (n < 0) return fail(EEGNET_EINVAL, "n must be >= 0");
    if (n == 0) return 0;
    if (int r = check_ptrs(x, "x", out, "out")) return r;
    ensure_attrs();
    const size_t lds = (size_t)(g.C * g.RS + NWB * (g.K1 + 1)) * 4;
    if (lds > (size_t)LDS_MAX) return fail(EEGNET_EINVAL, "eegnet_x_stats: dims need %zu B of LDS", lds);
    const dim3 grid((unsigned)std::min<int64_t>(n, (int64_t)device_cus() * WGPC));
    hipStream_t s = (hipStream_t)stream;
    {
        PROF(KID_XSTATS);
        if (g.K1 == 32) hipLaunchKernelGGL(k_xstats<32>, grid, dim3(NTB), lds, s, g, (long long)n, x, out);
        else hipLaunchKernelGGL(k_xstats<64>, grid, dim3(NTB), lds, s, g, (long long)n, x, out);
    }
    LAUNCH_CHECK("k_xstats");
    return 0;
}

int eegnet_clamp_grads(const eegnet_dims* dims, float* grads, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g, false)) return r;
    if (!grads) return fail(EEGNET_EINVAL, "grads is NULL");
    hipStream_t s = (hipStream_t)stream;
    const int n = std::max(g.F2 * g.C, NCLS * g.NF);
    hipLaunchKernelGGL(k_clamp, dim3((n + 255) / 256), dim3(256), 0, s, g, grads);
    LAUNCH_CHECK("k_clamp");
    return 0;
}

#ifdef EEGNET_TRACE
// debug hook of the traced build: workgroup 0 dumps its first trial's s [F2P,T], a [F2P,T/4] and
// z [F2P,T/4] planes (fp32) into `buf` (NULL turns it off)
int eegnet_debug_bf16(float* buf) {
    g_bf16_dbg = buf;
    return 0;
}
#endif

const char* eegnet_last_error(void) { return g_err.c_str(); }

int eegnet_trace_enable(void* buf) {
    g_trace_buf = (unsigned long long*)buf;
    return 0;
}

size_t eegnet_dims_bytes(void) { return sizeof(eegnet_dims); }
size_t eegnet_fold_bytes(void) { return sizeof(eegnet_fold); }
int eegnet_abi_version(void) { return EEGNET_ABI_VERSION; }

size_t eegnet_trace_bytes(void) { return (size_t)8 * TR_MAXWG * TR_SLOTS * sizeof(unsigned long long); }

int eegnet_profile_enable(int on) {
    g_prof.mask = (unsigned)on;
    return 0;
}

int eegnet_profile_collect(char* names, int* counts, double* total_ms, int cap, int* n_out) {
    double tot[KID_COUNT] = {0};
    int cnt[KID_COUNT] = {0};
    for (auto& r : g_prof.recs) {
        hipEventSynchronize(r.b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, r.a, r.b);
        tot[r.kid] += ms;
        cnt[r.kid] += 1;
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.recs.clear();
    int n = 0;
    for (int k = 0; k < KID_COUNT && n < cap; ++k) {
        if (!cnt[k]) continue;
        if (names) { strncpy(names + 32 * n, kKernelNames[k], 31); names[32 * n + 31] = 0; }
        if (counts) counts[n] = cnt[k];
        if (total_ms) total_ms[n] = tot[k];
        ++n;
    }
    if (n_out) *n_out = n;
    return 0;
}

const char* eegnet_build_info(void) {
    return "libeegnet_hip: gfx950 (CDNA4), fp32 VALU FIR/Gram + f32 MFMA 16x16x4 GEMMs, "
           "5-pass restructured EEGNet train step, 1024-thread row-per-wave workgroups, "
           "in-kernel ticketed fp64 reductions + finalize";
}

}  // extern "C"

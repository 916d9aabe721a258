"""Ablation builds of the cost kernel (timing experiments only; results are wrong).

    python scripts/ablate.py            # writes build_exp/libhq_<name>.so
    python scripts/profile_eval.py --lib build_exp/libhq_novfma.so

Each variant is hq_kernels.hip with one part of cost_tile_kernel removed by a
string patch on a copy (the product source is never modified); the delta
against "base" is that part's share of the kernel time (DESIGN.md
"Performance log").
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hybridquantization_amd", "csrc")
OUT = os.path.join(ROOT, "build_exp")

PATCHES = {
    "base": [],
    # vertical taps -> one multiply
    "novfma": [("            for (int y = 0; y < RV; ++y) acc[y] = fmaf(o[y + t], k, acc[y]);",
                "            for (int y = 0; y < RV; ++y) if (t == THI) acc[y] = o[y + t] * k;")],
    # horizontal taps -> one multiply
    "nohfma": [("            for (int xo = 0; xo < 4; ++xo) acc[xo] = fmaf(in[xo + t], k, acc[xo]);",
                "            for (int xo = 0; xo < 4; ++xo) if (t == THI) acc[xo] += in[xo + t] * k;")],
    # gather without the index dependency (same number of LDS reads)
    "nogather": [("            const float4 v = s_opp[s_idx[(gr * RV + r) * RW + c] * OPP_REP + copy];",
                  "            const float4 v = s_opp[((c + r) & 255) * OPP_REP + copy];")],
    # no Opp->Lab / dE
    "nolab": [("                const float3 lab = opp2lab_fast(acc0[xo], acc1[xo], acc2[xo], a.inv_illum[0],\n"
               "                                                a.inv_illum[1], a.inv_illum[2]);\n"
               "                const float e = delta_e<DE>(Ls[xo], As[xo], Bs[xo], lab.x, lab.y, lab.z);",
               "                const float e = acc0[xo] + acc1[xo] + acc2[xo] + Ls[xo] + As[xo] + Bs[xo];")],
    # index rows not loaded from HBM (synthetic bytes)
    "noidxload": [("            const uint32_t lo = src[0], hi = src[1];",
                   "            const uint32_t lo = (uint32_t)(e + (int)(intptr_t)src) * 2654435761u, hi = lo ^ 0x5bd1e995u;")],
    # opponent table not loaded (synthetic)
    "nooppload": [("        s_opp[e] = a.opp[(int64_t)p * kMaxK + e / OPP_REP];",
                   "        s_opp[e] = make_float4(e * 1e-3f, p * 1e-3f, 0.5f, 0.f);")],
    # LabRef not loaded
    "nolabload": [("            labL[h] = *reinterpret_cast<const float4*>(a.labL + off);\n"
                   "            labA[h] = *reinterpret_cast<const float4*>(a.labA + off);\n"
                   "            labB[h] = *reinterpret_cast<const float4*>(a.labB + off);",
                   "            labL[h] = make_float4(off * 1e-9f, 1.f, 2.f, 3.f);")],
    # gather address uniform over the wave (LDS broadcast: no bank conflicts)
    "gatherbcast": [("            const float4 v = s_opp[s_idx[(gr * RV + r) * RW + c] * OPP_REP + copy];",
                     "            const float4 v = s_opp[((gr * RV + r) & 255) * OPP_REP + copy];")],
    # H reads at a wave-uniform address (broadcast)
    "hreadbcast": [("        const float4* src = &s_v4[(y * RW) / 4 + j];\n        float acc0[4], acc1[4], acc2[4];\n        hpass_all<HALF, TH, RW, TRIM>(src, taps, acc0, acc1, acc2);\n        const int gy = y0 + y, gx0 = x0 + 4 * j;\n        if (gy < g.r1 && gx0 < g.W) {\n            const float4 L4",
                    "        const float4* src = &s_v4[(tid >> 6) * 8];\n        float acc0[4], acc1[4], acc2[4];\n        hpass_all<HALF, TH, RW, TRIM>(src, taps, acc0, acc1, acc2);\n        const int gy = y0 + y, gx0 = x0 + 4 * j;\n        if (gy < g.r1 && gx0 < g.W) {\n            const float4 L4")],
}
# H pass with separate accumulators for even and odd taps (4 independent chains)
PATCHES["hsplit"] = [(
    "            for (int xo = 0; xo < 4; ++xo) acc[xo] = fmaf(in[xo + t], k, acc[xo]);",
    "            for (int xo = 0; xo < 4; ++xo) { if (t & 1) acc2[xo] = fmaf(in[xo + t], k, acc2[xo]); else acc[xo] = fmaf(in[xo + t], k, acc[xo]); }"),
    ("        float in[4 * NQ];\n", "        float in[4 * NQ];\n        float acc2[4] = {0.f, 0.f, 0.f, 0.f};\n"),
    ("            for (int xo = 0; xo < 4; ++xo) { if (t & 1) acc2[xo] = fmaf(in[xo + t], k, acc2[xo]); else acc[xo] = fmaf(in[xo + t], k, acc[xo]); }\n        }\n",
     "            for (int xo = 0; xo < 4; ++xo) { if (t & 1) acc2[xo] = fmaf(in[xo + t], k, acc2[xo]); else acc[xo] = fmaf(in[xo + t], k, acc[xo]); }\n        }\n#pragma unroll\n        for (int xo = 0; xo < 4; ++xo) acc[xo] += acc2[xo];\n")]
# extra compiler flags per variant
FLAGS = {"noslp": [], "noslp_hsplit": []}  # -fno-slp-vectorize is now the product flag
PATCHES["noslp"] = []
PATCHES["noslp_hsplit"] = PATCHES["hsplit"]
# per-phase s_memtime stamps of cost_tile_kernel, summed over waves (hq_debug_phases)
PHASES_DECL = ("// VMODE: 0 = V items of RV rows on VALU",
               "__device__ unsigned long long g_phase[256 * 8];\n"
               "#define HQ_STAMP(k) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); "
               "if ((tid & 63) == 0) atomicAdd(&g_phase[(blockIdx.x & 255) * 8 + (k)], _t - _tp); _tp = _t; } while (0)\n"
               "// VMODE: 0 = V items of RV rows on VALU")
PATCHES["phases"] = [
    PHASES_DECL,
    ("    const int p = w % P_, tile = w / P_, tid = threadIdx.x;\n",
     "    const int p = w % P_, tile = w / P_, tid = threadIdx.x;\n    unsigned long long _tp = __builtin_amdgcn_s_memtime();\n"),
    ("    }\n    __syncthreads();\n\n    // ---- vertical pass:",
     "    }\n    HQ_STAMP(0);\n    __syncthreads();\n    HQ_STAMP(1);\n\n    // ---- vertical pass:"),
    ("    __syncthreads();\n\n    // ---- horizontal pass + Lab + dE",
     "    HQ_STAMP(2);\n    __syncthreads();\n    HQ_STAMP(3);\n\n    // ---- horizontal pass + Lab + dE"),
    ("    sum = wave_sum_to_lane63(sum);\n", "    HQ_STAMP(4);\n    sum = wave_sum_to_lane63(sum);\n"),
    ("        a.partial[(int64_t)p * a.ntiles + tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);\n}\n\n// ----------------------------------------------------------------------------\n// cost_persist",
     "        a.partial[(int64_t)p * a.ntiles + tile] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);\n    HQ_STAMP(5);\n    if ((tid & 63) == 0) atomicAdd(&g_phase[(blockIdx.x & 255) * 8 + 7], 1ull);\n}\n\n// ----------------------------------------------------------------------------\n// cost_persist"),
]
APPEND = {"phases": """
extern "C" int hq_debug_phases(unsigned long long* out, int reset) {
    static unsigned long long buf[256 * 8];
    if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(hq::g_phase), sizeof buf) != hipSuccess) return 1;
    for (int k = 0; k < 8; ++k) {
        out[k] = 0;
        for (int i = 0; i < 256; ++i) out[k] += buf[i * 8 + k];
    }
    if (reset) {
        for (auto& v : buf) v = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(hq::g_phase), buf, sizeof buf) != hipSuccess) return 1;
    }
    return 0;
}
"""}
# assign_batch: first candidate only (no candidate loop / slow path)
PATCHES["a_noloop"] = [(
    "            const int k = argmin_from_entry<REP>(r[j], gv[j], b[j], e[j], li[j], s_pal, copy, lvl1p,\n                                                 a.G2, a.K);",
    "            const int k = (int)((e[j].x >> 8) & 0xff) + (li[j] ? 0 : (int)s_pal[0].w);")]
# assign_batch: cell entry from a fixed cell (no RGB -> lookup dependency, L2-hot)
PATCHES["a_fixedcell"] = [(
    "            li[j] = lvl2_lookup(r[j], gv[j], b[j], lvl2p, a.G2, exh_pal || qb + 64 * j >= a.n_ext, e[j]);",
    "            li[j] = lvl2_lookup(0.5f, 0.5f, 0.5f + 1e-9f * r[j], lvl2p, a.G2, exh_pal || qb + 64 * j >= a.n_ext, e[j]);")]
# assign_pipe: first candidate only
PATCHES["p_noloop"] = [(
    """            const int k = argmin_from_entry<1>(xr[h], xg[h], xb[h], E[h][pp], in_[h] && !exh_pal[pp],
                                               s_pal + pp * a.K, 0,
                                               a.lvl1 + (int64_t)pq * a.lvl1_pitch, G2, a.K);""",
    """            const int k = (int)((E[h][pp].x >> 8) & 0xff) + (in_[h] ? 0 : (int)s_pal[0].w);""")]
# cost_pair: LabRef loaded after the vertical pass (register pressure during V)
_LAB_BLOCK_START = "    float labv[2][3][HR];\n"
_LAB_BLOCK_END = "    __syncthreads();\n\n    // ---- vertical pass (row-pair output layout)"


def _lab_after_v(src):
    i = src.index(_LAB_BLOCK_START)
    j = src.index(_LAB_BLOCK_END, i)
    block = src[i:j]
    src = src[:i] + src[j:]
    anchor = "    __syncthreads();\n\n    // ---- horizontal pass over the row pair + Lab + dE ----\n"
    k = src.index(anchor)
    return src[:k] + block + src[k:]


TRANSFORMS = {"p_labafter": _lab_after_v}
PATCHES["p_labafter"] = []
# cost_pair: H-pass window reads at a wave-uniform address (LDS broadcast; results wrong)
PATCHES["p_hbcast"] = [("        hpass_pair_all<HALF, TH, RW, HR, TRIM>(&s_vq[(m * RW + HR * jr) / 2], taps, acc0, acc1, acc2);",
                        "        hpass_pair_all<HALF, TH, RW, HR, TRIM>(&s_vq[(tid >> 6) * 8], taps, acc0, acc1, acc2);")]
# cost_pair: V-pass gathers at a wave-uniform table entry (results wrong)
PATCHES["p_gbcast"] = [("            const float4 v = s_opp[s_idx[(gr * RV + r) * RW + c]];\n            o0[r] = v.x;",
                        "            const float4 v = s_opp[(gr * RV + r + (s_idx[(gr * RV + r) * RW + c] >> 7)) & 255];\n            o0[r] = v.x;")]
PATCHES["p_bothbcast"] = PATCHES["p_hbcast"] + PATCHES["p_gbcast"]
# cost_chan: 5 workgroups per CU (96 VGPRs)
PATCHES["c_occ5"] = [("__launch_bounds__(256, 6) void cost_chan_kernel", "__launch_bounds__(256, 5) void cost_chan_kernel")]


def _chan_lab_late(src):
    i = src.index("void cost_chan_kernel(")
    a = src.index("    float labv[2][3][HR];\n", i)
    b = src.index("    __syncthreads();\n", a)
    block = src[a:b]
    src = src[:a] + src[b:]
    anchor = "    __syncthreads();\n\n    double sum = 0.0;\n"
    k = src.index(anchor, i)
    return src[:k] + block + src[k:]


TRANSFORMS["c_lablate"] = _chan_lab_late
PATCHES["c_lablate"] = []  # (now the product layout; kept for old revisions)
# assign_pipe at 8 / 6 waves per SIMD (64 / 80 VGPRs)
PATCHES["a_lb8"] = [("__launch_bounds__(256) void assign_pipe_kernel", "__launch_bounds__(256, 8) void assign_pipe_kernel")]
PATCHES["a_lb6"] = [("__launch_bounds__(256) void assign_pipe_kernel", "__launch_bounds__(256, 6) void assign_pipe_kernel")]
# cost_mfma / cost_mm: MFMA tap fragments loaded at a wave-uniform address (results wrong)
PATCHES["m_fragbcast"] = [("    const uint4* frag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]",
                           "    const uint4* frag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + (lane >> 6);")]
PATCHES["mm_fragbcast"] = [("    const uint4* vfrag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + lane;  // [trim][stack][hi,lo][lane]",
                            "    const uint4* vfrag = a.vfrag16 + (TRIM ? 4 * 2 * 64 : 0) + (lane >> 6);"),
                           ("    const uint4* hfrag = a.hfrag16 + (TRIM ? 7 * 2 * 64 : 0) + lane;  // [trim][filter][hi,lo][lane]",
                            "    const uint4* hfrag = a.hfrag16 + (TRIM ? 7 * 2 * 64 : 0) + (lane >> 6);")]
PATCHES["skeleton"] = PATCHES["novfma"] + PATCHES["nohfma"] + PATCHES["nolab"]
PATCHES["skeleton_bcast"] = PATCHES["skeleton"] + PATCHES["gatherbcast"]


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(os.path.join(CSRC, "hq_kernels.hip")).read()
    names = sys.argv[1:] or list(PATCHES)
    for name in names:
        s = src
        if name.startswith("git:"):  # git:<rev> = that revision's kernels (A/B baseline)
            rev = name[4:]
            s = subprocess.check_output(["git", "-C", ROOT, "show",
                                         f"{rev}:hybridquantization_amd/csrc/hq_kernels.hip"]).decode()
            name = "rev_" + rev
            PATCHES[name] = []
        for old, new in PATCHES[name]:
            if old not in s:
                sys.exit(f"{name}: patch anchor not found")
            s = s.replace(old, new)
        if name in TRANSFORMS:
            s = TRANSFORMS[name](s)
        s += APPEND.get(name, "")
        path = os.path.join(OUT, f"hq_kernels_{name}.hip")
        open(path, "w").write(s)
        obj = os.path.join(OUT, f"hq_kernels_{name}.o")
        flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-I/opt/rocm/include",
                 "-I" + CSRC, "-munsafe-fp-atomics", "-fno-slp-vectorize", *FLAGS.get(name, [])]
        subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", path, "-o", obj])
        so = os.path.join(OUT, f"libhq_{name}.so")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", obj,
                               os.path.join(CSRC, "hq_runtime.o"), os.path.join(CSRC, "hq_host.o"),
                               "-shared", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib",
                               "-o", so])
        print("built", so)


if __name__ == "__main__":
    main()

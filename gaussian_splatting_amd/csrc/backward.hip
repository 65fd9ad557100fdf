// backward.hip -- per-Gaussian backward.
//
//   gauss_reduce_kernel (one lane per Gaussian): sums each Gaussian's
//     per-(tile) gradient records.  They are contiguous per Gaussian and the
//     Gaussians' ranges follow each other, so consecutive lanes read
//     consecutive memory and the sum is deterministic -- no atomics.
//   gauss_bwd_kernel (one wave per 64 Gaussians):
//     - computeCov2DCUDA (CR/backward.cu:153-290) including the tail that the
//       vendored file truncates (dL/dcov3D and dL/dmean3D through the EWA
//       projection, the clamp masks and the inverse-depth term), derived in
//       DESIGN.md "Backward conventions";
//     - preprocessCUDA (CR/backward.cu:372-429): screen-space mean -> 3-D mean,
//       SH colour backward (:12-146) and scale/rotation backward (:296-365).
//     The 64 SH rows of the wave (64 x 192 B when M = 16) are staged through LDS
//     so both the global read of the coefficients and the write of dL/dSH are
//     fully coalesced 16-byte accesses; the SH backward streams one coefficient
//     at a time instead of holding 48 floats in registers.
// Every output row is written, zeros included, so the host never memsets the
// gradient tensors (the reference zero-fills all of them first,
// RI/rasterize_points.cu:186-195).
#include "kernels.h"

namespace gsr {

// ---- 1. segmented sums of the per-instance records ------------------------------
// One wave per 64 consecutive Gaussians.  Their records form one contiguous range
// [E0, E1) (record index = rec_start[g] + k, k = the tile's row-major index in g's
// rectangle).  A record exists iff its content bit is set (render.hip writes records only for
// entries with a gradient term; the bits are zeroed by the forward's K3, binning.hip) -- 5M@4K:
// 7.6M records of 114.7M instances, the rest behind saturated pixels.  Per window of 1024
// positions the positions of the records are compacted into an LDS list (per-lane popcounts of
// the set bits, a wave prefix sum, each lane writing its own positions), and the list is reduced
// 64 RECORDS at a time: at 1M@1080p a wave's ~508 instance positions hold ~80 records, two
// groups.  A Gaussian's records are its slots [r0, r1) of the list (counted from the bits below
// its range start and end); each group is summed by a segmented scan over the wave (DPP row
// shifts and row broadcasts, the add masked where the source lane belongs to another Gaussian),
// which leaves each Gaussian's group total in the last lane of its run, handed to the owner lane
// through LDS.  A fixed order: the result does not depend on scheduling.  The records of a
// window's next group are requested before its current group is reduced, the radius is read at
// the start, and the LDS hand-offs are wave-local (the workgroup is one wave).
constexpr int kRecStride = 12;  // floats per Gaussian in the LDS hand-off of group totals (10 used), 48 B
__device__ __forceinline__ void reduce_sync() {
    wave_lds_sync();
}
__device__ __forceinline__ uint64_t byte_flags(uint64_t x) {  // each nonzero byte -> 0x01, zero -> 0x00
    x |= x >> 4;
    x |= x >> 2;
    x |= x >> 1;
    return x & 0x0101010101010101ull;
}
__device__ __forceinline__ void reduce_records_compact(int P, int g0, const uint32_t* __restrict__ rec_start,
                                                       const uint32_t* __restrict__ tiles_touched,
                                                       const GradRecs& recs, float* s_rec, float4& sa, float4& sb,
                                                       float2& sc) {
    const int lane = threadIdx.x;
    const int g = g0 + lane;
    const bool valid = g < P;
    const int g_last = min(g0 + 63, P - 1);
    const uint32_t E0 = rec_start[g0];
    const uint32_t E1 = rec_start[g_last] + tiles_touched[g_last];
    const uint32_t n = valid ? tiles_touched[g] : 0u;
    const uint32_t my0 = valid ? rec_start[g] : E1;
    const uint32_t my1 = my0 + n;
    sa = make_float4(0.f, 0.f, 0.f, 0.f);
    sb = sa;
    sc = make_float2(0.f, 0.f);
    __shared__ uint16_t s_list[1024];  // the window's record positions, as offsets from its first byte
    __shared__ uint32_t s_mark[64];
    float4* part = reinterpret_cast<float4*>(s_rec);  // [64][3] float4: a Gaussian's group total
    for (uint32_t wa = E0 & ~15u; wa < E1; wa += 1024u) {  // uniform
        // content bytes [wa, wa + 1024): lane l holds wa + 16 l .. + 15, masked to [E0, E1)
        const uint32_t p = wa + 16u * (uint32_t)lane;
        // (flag bits: this lane's 16 positions are half of one 32-bit word, wa being a multiple of 16)
        uint32_t m16 = 0;
        if (p < E1) {
            m16 = (reinterpret_cast<const uint32_t*>(recs.flag)[p >> 5] >> (p & 16u)) & 0xffffu;
            const uint32_t k = E1 - p;  // positions of this lane below E1
            if (k < 16) m16 &= (1u << k) - 1u;
            if (p < E0) m16 &= 0xffffu << (E0 - p);  // (first window, lane 0 only) the previous wave's
        }
        const uint32_t c = (uint32_t)__popc(m16);
        const uint32_t incl = wave_incl_sum(c), off = incl - c;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);  // records in the window
        if (R == 0) continue;  // uniform
        wave_lds_sync();  // the previous window's readers are done (in-order LDS)
        {
            uint32_t k = off;
            for (uint32_t t = m16; t; t &= t - 1) s_list[k++] = (uint16_t)(16 * lane + __builtin_ctz(t));
        }
        wave_lds_sync();
        auto slots_below = [&](uint32_t q) -> uint32_t {
            const uint32_t d = q <= wa ? 0u : min(q - wa, 1024u);
            const int L = (int)min(d >> 4, 63u);
            const uint32_t offL = (uint32_t)__shfl((int)off, L), mL = (uint32_t)__shfl((int)m16, L);
            const uint32_t b = d - 16u * (uint32_t)L;  // positions of lane L below q (16: all of them)
            return offL + (uint32_t)__popc(mL & (b >= 16 ? 0xffffu : (1u << b) - 1u));
        };
        // (both calls on every lane: slots_below shuffles across lanes, so it must not sit in a branch)
        const uint32_t r0 = slots_below(my0), r1e = slots_below(my1), r1 = n ? r1e : r0;
        const bool mine = r1 > r0;
        // the next group's records are requested before this group is reduced (one latency per window
        // instead of one per group)
        float4 xn = make_float4(0.f, 0.f, 0.f, 0.f), yn = xn;
        float2 zn = make_float2(0.f, 0.f);
        if ((uint32_t)lane < R) {
            const uint32_t e = wa + (uint32_t)s_list[lane];
            xn = recs.a[(size_t)kRecAB * e];
            yn = recs.b[(size_t)kRecAB * e];
            zn = recs.c[(size_t)kRecC * e];
        }
        for (uint32_t k0 = 0; k0 < R; k0 += 64) {  // uniform: 64 records at a time
            const uint32_t k = k0 + (uint32_t)lane;
            const bool has = k < R;
            const float4 x = xn, y = yn;
            const float2 z = zn;
            if (k + 64 < R) {
                const uint32_t e = wa + (uint32_t)s_list[k + 64];
                xn = recs.a[(size_t)kRecAB * e];
                yn = recs.b[(size_t)kRecAB * e];
                zn = recs.c[(size_t)kRecC * e];
            } else {  // (lanes past the window's records: zeros, as unloaded lanes always held)
                xn = yn = make_float4(0.f, 0.f, 0.f, 0.f);
                zn = make_float2(0.f, 0.f);
            }
            // owner of slot k: the largest lane with records whose first slot is <= k
            const unsigned long long st = __ballot(mine && r0 < k0);
            const uint32_t carry = st ? 64u - (uint32_t)__clzll((long long)st) : 0u;
            s_mark[lane] = 0u;
            wave_lds_sync();
            if (mine && r0 >= k0 && r0 < k0 + 64) s_mark[r0 - k0] = (uint32_t)lane + 1u;
            wave_lds_sync();
            const uint32_t m = max(wave_incl_max(s_mark[lane]), carry);
            wave_lds_sync();
            const int owner = has && m ? (int)m - 1 : -1;
            const uint32_t o0 = (uint32_t)__shfl((int)r0, owner < 0 ? 0 : owner);
            const int seg0 = has ? (o0 > k0 ? (int)(o0 - k0) : 0) : lane;
            const int r = lane & 15, row = lane >> 4;
            const float m1 = lane - 1 >= seg0 && r >= 1 ? 1.f : 0.f, m2 = lane - 2 >= seg0 && r >= 2 ? 1.f : 0.f,
                        m4 = lane - 4 >= seg0 && r >= 4 ? 1.f : 0.f, m8 = lane - 8 >= seg0 && r >= 8 ? 1.f : 0.f,
                        mb15 = (row & 1) && row * 16 - 1 >= seg0 ? 1.f : 0.f,
                        mb31 = row >= 2 && 31 >= seg0 ? 1.f : 0.f;
            float v[10] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y};
#pragma unroll
            for (int i = 0; i < 10; i++) {
                v[i] = fmaf(dpp_f32<0x111, 0xf, true>(v[i]), m1, v[i]);
                v[i] = fmaf(dpp_f32<0x112, 0xf, true>(v[i]), m2, v[i]);
                v[i] = fmaf(dpp_f32<0x114, 0xf, true>(v[i]), m4, v[i]);
                v[i] = fmaf(dpp_f32<0x118, 0xf, true>(v[i]), m8, v[i]);
                v[i] = fmaf(dpp_f32<0x142, 0xa, false>(v[i]), mb15, v[i]);
                v[i] = fmaf(dpp_f32<0x143, 0xc, false>(v[i]), mb31, v[i]);
            }
            const int next_owner = __shfl_down(owner, 1);
            if (owner >= 0 && (lane == 63 || next_owner != owner)) {  // the run's last lane hands it over
                part[owner * 3 + 0] = make_float4(v[0], v[1], v[2], v[3]);
                part[owner * 3 + 1] = make_float4(v[4], v[5], v[6], v[7]);
                part[owner * 3 + 2] = make_float4(v[8], v[9], 0.f, 0.f);
            }
            reduce_sync();
            if (max(r0, k0) < min(r1, k0 + 64)) {  // this Gaussian has records in the group
                const float4 pp = part[lane * 3 + 0], q = part[lane * 3 + 1], ww = part[lane * 3 + 2];
                sa.x += pp.x; sa.y += pp.y; sa.z += pp.z; sa.w += pp.w;
                sb.x += q.x; sb.y += q.y; sb.z += q.z; sb.w += q.w;
                sc.x += ww.x; sc.y += ww.y;
            }
            reduce_sync();
        }
    }
}

__global__ void __launch_bounds__(64) gauss_reduce_kernel(int P, const uint32_t* __restrict__ rec_start,
                                                          const uint32_t* __restrict__ tiles_touched,
                                                          GradRecs recs, GradRecs sums, uint32_t* __restrict__ flags,
                                                          const int* __restrict__ radii,
                                                          const uint8_t* __restrict__ clamped,
                                                          uint32_t* __restrict__ live,
                                                          uint32_t* __restrict__ live_count, uint32_t live_cap) {
    __shared__ __attribute__((aligned(16))) float s_rec[64 * kRecStride];
    const int g = blockIdx.x * 64 + (int)threadIdx.x;
    const int rad = g < P ? radii[g] : 0;  // requested with the range loads, not after the reduction
    float4 sa, sb;
    float2 sc;
    reduce_records_compact(P, blockIdx.x * 64, rec_start, tiles_touched, recs, s_rec, sa, sb, sc);
    // a Gaussian with a gradient (gauss_bwd's condition)
    const bool lv = g < P && rad > 0 &&
                    ((sa.x != 0.f) | (sa.y != 0.f) | (sa.z != 0.f) | (sa.w != 0.f) | (sb.x != 0.f) |
                     (sb.y != 0.f) | (sb.z != 0.f) | (sb.w != 0.f) | (sc.x != 0.f) | (sc.y != 0.f));
    // With a live list (single view) gauss_bwd reads the sums of the listed Gaussians only, so the
    // other ~87% (zeros) are not written; a view block (flags) or the dense backward reads every row.
    if (g < P && (!live || flags || lv)) {
        sums.a[g] = sa;
        sums.b[g] = sb;
        sums.c[g] = sc;
    }
    // view-block flag word (gauss_bwd_views_kernel): bit 0 visible, bits 1-3 the SH clamp mask
    if (g < P && flags) flags[g] = (rad > 0 ? 1u : 0u) | ((uint32_t)(clamped[g] & 7u) << 1);
    if (live) {
        // append them to the live list: one atomic per wave; the list order varies from run to run,
        // each entry's result does not
        const unsigned long long m = __ballot(lv);
        if (m) {  // uniform
            const int lane = threadIdx.x;
            const uint32_t shard = blockIdx.x % kLiveShards;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&live_count[shard * kLiveCntStride], (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, 0);
            if (lv) live[(size_t)shard * live_cap + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)g;
        }
    }
}

hipError_t launch_gauss_reduce(int P, const GeomState& g, const GradRecs& recs, const GradRecs& sums,
                               uint32_t* flags, const int* radii, uint32_t* live, uint32_t* live_count,
                               hipStream_t stream) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_reduce_kernel, dim3((P + 63) / 64), dim3(64), 0, stream, P, g.rec_start, g.tiles_touched,
                       recs, sums, flags, radii, g.clamped, live, live_count, live_list_cap((uint32_t)P));
    return hipGetLastError();
}

// ---- 1b. atomic backward ----------------------------------------------------------
// render_bwd ("bwd_atomic") added every instance's sums into its Gaussian's accumulator row and set
// the Gaussian's touched bit; gauss_bwd_touched_kernel (section 3) reads the rows of the touched
// Gaussians and restores them to zero, gauss_live_views (below) fills a view block from them.

// The atomic backward into a view block (gsr_rasterize_backward_screen, multi-GPU view exchange): one lane
// per Gaussian writes its dense sums -- its accumulator row if its touched bit is set (the row then zeroed),
// zeros otherwise -- and its flag word, as gauss_reduce does for a view block; the words it read are cleared.
__global__ void __launch_bounds__(64) gauss_live_views_kernel(int P, uint32_t* __restrict__ touched,
                                                              float4* __restrict__ acc, const int* __restrict__ radii,
                                                              const uint8_t* __restrict__ clamped, GradRecs sums,
                                                              uint32_t* __restrict__ flags) {
    const int lane = threadIdx.x;
    const uint32_t g = blockIdx.x * 64u + (uint32_t)lane;
    if (g >= (uint32_t)P) return;
    const uint32_t w = touched[g >> 5];
    const bool lv = (w >> (g & 31u)) & 1u;
    float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra, rc = ra;
    float4* row = acc + (size_t)g * kAccRow4;
    if (lv) {
        ra = row[0];
        rb = row[1];
        rc = row[2];
    }
    const int rad = radii[g];
    const uint8_t cm = clamped[g];
    sums.a[g] = ra;
    sums.b[g] = rb;
    sums.c[g] = make_float2(rc.x, rc.y);
    flags[g] = (rad > 0 ? 1u : 0u) | ((uint32_t)(cm & 7u) << 1);
    if (lv) row[0] = row[1] = row[2] = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((lane & 31) == 0 && w) touched[g >> 5] = 0u;  // (after every lane's read: the stores depend on w)
}

hipError_t launch_gauss_live_views(int P, uint32_t* touched, float4* acc, const int* radii, const uint8_t* clamped,
                                   const GradRecs& sums, uint32_t* flags, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_live_views_kernel, dim3((uint32_t)(((size_t)P + 63) / 64)), dim3(64), 0, stream, P, touched,
                       acc, radii, clamped, sums, flags);
    return hipGetLastError();
}

// ---- 2. SH colour backward, one coefficient at a time ---------------------------
// Row accessors: coefficient k of this thread's Gaussian (3 floats).
struct ShLds {
    float* row;  // LDS row, padded stride
    __device__ float3 load(int k) const { return make_float3(row[3 * k], row[3 * k + 1], row[3 * k + 2]); }
    __device__ void store(int k, float3 v) const {
        row[3 * k] = v.x;
        row[3 * k + 1] = v.y;
        row[3 * k + 2] = v.z;
    }
};
struct ShGlobal {
    ShAddr src;
    ShGradAddr dst;
    int idx;
    __device__ float3 load(int k) const {
        const float* c = src.coef(idx, k);
        return make_float3(c[0], c[1], c[2]);
    }
    __device__ void store(int k, float3 v) const {
        float* c = dst.coef(idx, k);
        c[0] = v.x;
        c[1] = v.y;
        c[2] = v.z;
    }
};

// For each coefficient k < (deg+1)^2: dL/dsh_k = B_k(dir) * g, and
// d(colour . g)/d(dir) += grad B_k(dir) * (sh_k . g)  (CR/backward.cu:43-127).
// Coefficients k >= (deg+1)^2 (up to M) get zero gradients.
template <class Acc>
__device__ __forceinline__ void sh_backward(const Acc& acc, int deg, int M, float x, float y, float z, float3 g,
                                            float& ddx, float& ddy, float& ddz) {
    ddx = ddy = ddz = 0.f;
    auto term = [&](int k, float B, float bx, float by, float bz) {
        const float3 s = acc.load(k);
        const float sg = s.x * g.x + s.y * g.y + s.z * g.z;
        ddx += bx * sg;
        ddy += by * sg;
        ddz += bz * sg;
        acc.store(k, make_float3(B * g.x, B * g.y, B * g.z));
    };
    term(0, SH_C0, 0.f, 0.f, 0.f);
    int K = 1;
    if (deg > 0) {
        term(1, -SH_C1 * y, 0.f, -SH_C1, 0.f);
        term(2, SH_C1 * z, 0.f, 0.f, SH_C1);
        term(3, -SH_C1 * x, -SH_C1, 0.f, 0.f);
        K = 4;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            term(4, SH_C2_0 * xy, SH_C2_0 * y, SH_C2_0 * x, 0.f);
            term(5, SH_C2_1 * yz, 0.f, SH_C2_1 * z, SH_C2_1 * y);
            term(6, SH_C2_2 * (2.f * zz - xx - yy), SH_C2_2 * -2.f * x, SH_C2_2 * -2.f * y, SH_C2_2 * 4.f * z);
            term(7, SH_C2_3 * xz, SH_C2_3 * z, 0.f, SH_C2_3 * x);
            term(8, SH_C2_4 * (xx - yy), SH_C2_4 * 2.f * x, SH_C2_4 * -2.f * y, 0.f);
            K = 9;
            if (deg > 2) {
                term(9, SH_C3_0 * y * (3.f * xx - yy), SH_C3_0 * 6.f * xy, SH_C3_0 * 3.f * (xx - yy), 0.f);
                term(10, SH_C3_1 * xy * z, SH_C3_1 * yz, SH_C3_1 * xz, SH_C3_1 * xy);
                term(11, SH_C3_2 * y * (4.f * zz - xx - yy), SH_C3_2 * -2.f * xy, SH_C3_2 * (-3.f * yy + 4.f * zz - xx),
                     SH_C3_2 * 8.f * yz);
                term(12, SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy), SH_C3_3 * -6.f * xz, SH_C3_3 * -6.f * yz,
                     SH_C3_3 * 3.f * (2.f * zz - xx - yy));
                term(13, SH_C3_4 * x * (4.f * zz - xx - yy), SH_C3_4 * (-3.f * xx + 4.f * zz - yy), SH_C3_4 * -2.f * xy,
                     SH_C3_4 * 8.f * xz);
                term(14, SH_C3_5 * z * (xx - yy), SH_C3_5 * 2.f * xz, SH_C3_5 * -2.f * yz, SH_C3_5 * (xx - yy));
                term(15, SH_C3_6 * x * (xx - 3.f * yy), SH_C3_6 * 3.f * (xx - yy), SH_C3_6 * -6.f * xy, 0.f);
                K = 16;
            }
        }
    }
    for (int k = K; k < M; k++) acc.store(k, make_float3(0.f, 0.f, 0.f));
}

__device__ __forceinline__ void store3(float* p, int i, float x, float y, float z) {
    p[3 * i] = x;
    p[3 * i + 1] = y;
    p[3 * i + 2] = z;
}

constexpr int kShStride = 52;  // padded LDS row stride: conflict-free ds_read/write_b128

// ---- per-view gradient math (one Gaussian, one view) ----------------------------
// computeCov2DCUDA with its re-derived tail, the screen-space mean chain, the SH colour
// backward and the scale/rotation backward, from the view's summed render gradients.  The one
// copy of this math: gauss_bwd_kernel runs it once per Gaussian, gauss_bwd_views_kernel once
// per (Gaussian, view).  The outputs leave through the caller's sink as soon as each is formed
// (the single-view kernel stores them there and then, which keeps its register peak down; the
// multi-view kernel sums them over the views).  Sink interface:
//   dop(float)  dcov(const float (&)[6])  dmean(float3)  scale_rot(bool have, float3, float4)
//   sh_defer(float3 view vector, float3 masked colour gradient)   (kShDefer only)
struct ViewCam {
    const float* V;       // viewmatrix, 16 floats (column-major)
    const float* Pm;      // projmatrix
    const float* campos;  // 3
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int antialiasing, have_invdepth;
};
struct GaussIn {
    float3 mean;
    bool have_scales;
    float3 sc3;            // scales (when have_scales)
    float4 q;              // rotation (when have_scales)
    const float* cov3D;    // 6 floats, or null
    float scale_modifier;
    const float* opacity;  // the Gaussian's opacity (read by the AA chain only)
};
// SH colour backward of view_backward (when do_sh: the colours came from SH, not precomputed):
// now (through the accessor, adding the view-direction term to dL/dmean3D), or deferred (the
// caller runs it later from what sink.sh_defer receives, then stores dL/dmean3D itself).
enum { kShNow = 1, kShDefer = 2 };

// d(normalize(v))/dv applied to the direction gradient (dnormvdv, CR/auxiliary.h:129-139),
// added to dmean.
__device__ __forceinline__ void add_dir_grad(float3 v, float ddx, float ddy, float ddz, float3& dmean) {
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    dmean.x += ((sum2 - v.x * v.x) * ddx - v.y * v.x * ddy - v.z * v.x * ddz) * invsum32;
    dmean.y += (-v.x * v.y * ddx + (sum2 - v.y * v.y) * ddy - v.z * v.y * ddz) * invsum32;
    dmean.z += (-v.x * v.z * ddx - v.y * v.z * ddy + (sum2 - v.z * v.z) * ddz) * invsum32;
}

// SH colour backward for view vector v (mean - campos) and colour gradient g: dL/dSH through the
// accessor, the direction term added to dmean (CR/backward.cu:12-146).
template <class ShAcc>
__device__ __forceinline__ void sh_dir_backward(const ShAcc& sh, int D, int M, float3 v, float3 g, float3& dmean) {
    const float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    float ddx, ddy, ddz;
    sh_backward(sh, D, M, v.x / len, v.y / len, v.z / len, g, ddx, ddy, ddz);
    add_dir_grad(v, ddx, ddy, ddz, dmean);
}

template <int SHM, class ShAcc, class Sink>
__device__ __forceinline__ void view_backward(const ViewCam& c, const GaussIn& gi, float4 sa, float4 sb, float2 sc,
                                              uint8_t cm, bool do_sh, int D, int M, const ShAcc& sh, Sink& out) {
    const float3 dcol = make_float3(sa.x, sa.y, sa.z);
    const float dinvd = sa.w;
    const float m2x = sb.x, m2y = sb.y;
    float dop = sb.z;
    const float dca = sc.x, dcb = sb.w, dcc = sc.y;  // dL/dconic, the reference's convention
    // ---- computeCov2DCUDA
    const float* V = c.V;
    const float3 mean = gi.mean;
    float3 t = xform_point_4x3(mean, V);
    const float limx = 1.3f * c.tan_fovx, limy = 1.3f * c.tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
    const float fx = c.focal_x, fy = c.focal_y;
    const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
    const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
    // A = J * Rv, rows A0 (x) and A1 (y); Rv rows (V0,V4,V8) (V1,V5,V9) (V2,V6,V10)
    const float A0[3] = {j00 * V[0] + j02 * V[2], j00 * V[4] + j02 * V[6], j00 * V[8] + j02 * V[10]};
    const float A1[3] = {j11 * V[1] + j12 * V[2], j11 * V[5] + j12 * V[6], j11 * V[9] + j12 * V[10]};

    float cov[6];
    const float3 sc3 = gi.sc3;
    const float4 q = gi.q;
    if (gi.cov3D) {
        for (int k = 0; k < 6; k++) cov[k] = gi.cov3D[k];
    } else {
        const float r_ = q.x, x = q.y, y = q.z, z = q.w;
        const float sx = gi.scale_modifier * sc3.x, sy = gi.scale_modifier * sc3.y, sz = gi.scale_modifier * sc3.z;
        const float L00 = (1.f - 2.f * (y * y + z * z)) * sx, L01 = 2.f * (x * y - r_ * z) * sy,
                    L02 = 2.f * (x * z + r_ * y) * sz;
        const float L10 = 2.f * (x * y + r_ * z) * sx, L11 = (1.f - 2.f * (x * x + z * z)) * sy,
                    L12 = 2.f * (y * z - r_ * x) * sz;
        const float L20 = 2.f * (x * z - r_ * y) * sx, L21 = 2.f * (y * z + r_ * x) * sy,
                    L22 = (1.f - 2.f * (x * x + y * y)) * sz;
        cov[0] = L00 * L00 + L01 * L01 + L02 * L02;
        cov[1] = L00 * L10 + L01 * L11 + L02 * L12;
        cov[2] = L00 * L20 + L01 * L21 + L02 * L22;
        cov[3] = L10 * L10 + L11 * L11 + L12 * L12;
        cov[4] = L10 * L20 + L11 * L21 + L12 * L22;
        cov[5] = L20 * L20 + L21 * L21 + L22 * L22;
    }
    const float SA0[3] = {cov[0] * A0[0] + cov[1] * A0[1] + cov[2] * A0[2],
                          cov[1] * A0[0] + cov[3] * A0[1] + cov[4] * A0[2],
                          cov[2] * A0[0] + cov[4] * A0[1] + cov[5] * A0[2]};
    const float SA1[3] = {cov[0] * A1[0] + cov[1] * A1[1] + cov[2] * A1[2],
                          cov[1] * A1[0] + cov[3] * A1[1] + cov[4] * A1[2],
                          cov[2] * A1[0] + cov[4] * A1[1] + cov[5] * A1[2]};
    float c_xx = A0[0] * SA0[0] + A0[1] * SA0[1] + A0[2] * SA0[2];
    const float c_xy = A0[0] * SA1[0] + A0[1] * SA1[1] + A0[2] * SA1[2];
    float c_yy = A1[0] * SA1[0] + A1[1] * SA1[1] + A1[2] * SA1[2];

    constexpr float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (c.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float d_h = dop * *gi.opacity;
        dop = dop * h;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f : d_h / (2.f * h);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0.f, dL_dc_xy = 0.f, dL_dc_yy = 0.f;
    if (c.antialiasing) {
        // the reference's formula (CR/backward.cu:256-270), at the dilated x, y as written there
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float qd = w * w + w * (x + y) + x * y - z * z;
        const float denom_f = d_inside_root / (qd * qd);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    if (denom2inv != 0.f) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dca + 2.f * c_xy * c_yy * dcb + (denom - c_xx * c_yy) * dcc);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dcc + 2.f * c_xx * c_xy * dcb + (denom - c_xx * c_yy) * dca);
        dL_dc_xy += denom2inv * 2.f * (c_xy * c_yy * dca - (denom + 2.f * c_xy * c_xy) * dcb + c_xx * c_xy * dcc);
    }
    out.dop(dop);

    // tail: cov2D = A Sigma A^T  ->  dL/dcov3D (6 stored entries) and dL/dA
    const float ga = dL_dc_xx, gb = dL_dc_xy, gc = dL_dc_yy;
    float dcov[6];
    dcov[0] = A0[0] * A0[0] * ga + A0[0] * A1[0] * gb + A1[0] * A1[0] * gc;
    dcov[3] = A0[1] * A0[1] * ga + A0[1] * A1[1] * gb + A1[1] * A1[1] * gc;
    dcov[5] = A0[2] * A0[2] * ga + A0[2] * A1[2] * gb + A1[2] * A1[2] * gc;
    dcov[1] = 2.f * A0[0] * A0[1] * ga + (A0[0] * A1[1] + A0[1] * A1[0]) * gb + 2.f * A1[0] * A1[1] * gc;
    dcov[2] = 2.f * A0[0] * A0[2] * ga + (A0[0] * A1[2] + A0[2] * A1[0]) * gb + 2.f * A1[0] * A1[2] * gc;
    dcov[4] = 2.f * A0[2] * A0[1] * ga + (A0[1] * A1[2] + A0[2] * A1[1]) * gb + 2.f * A1[1] * A1[2] * gc;
    out.dcov(dcov);

    float dA0[3], dA1[3];
    for (int k = 0; k < 3; k++) {
        dA0[k] = 2.f * ga * SA0[k] + gb * SA1[k];
        dA1[k] = 2.f * gc * SA1[k] + gb * SA0[k];
    }
    const float dJ00 = dA0[0] * V[0] + dA0[1] * V[4] + dA0[2] * V[8];
    const float dJ02 = dA0[0] * V[2] + dA0[1] * V[6] + dA0[2] * V[10];
    const float dJ11 = dA1[0] * V[1] + dA1[1] * V[5] + dA1[2] * V[9];
    const float dJ12 = dA1[0] * V[2] + dA1[1] * V[6] + dA1[2] * V[10];
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -fx * tz2 * dJ02;
    const float dL_dty = y_grad_mul * -fy * tz2 * dJ12;
    float dL_dtz =
        -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * t.x) * tz3 * dJ02 + (2.f * fy * t.y) * tz3 * dJ12;
    if (c.have_invdepth) dL_dtz -= dinvd / (t.z * t.z);
    // transformVec4x3Transpose (CR/auxiliary.h:109-117)
    float3 dmean = make_float3(V[0] * dL_dtx + V[1] * dL_dty + V[2] * dL_dtz,
                               V[4] * dL_dtx + V[5] * dL_dty + V[6] * dL_dtz,
                               V[8] * dL_dtx + V[9] * dL_dty + V[10] * dL_dtz);

    // ---- screen-space mean -> 3-D mean through the projection (CR/backward.cu:403-420)
    const float* Pm = c.Pm;
    const float4 m_hom = xform_point_4x4(mean, Pm);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = m_hom.x * m_w * m_w, mul2 = m_hom.y * m_w * m_w;
    dmean.x += (Pm[0] * m_w - Pm[3] * mul1) * m2x + (Pm[1] * m_w - Pm[3] * mul2) * m2y;
    dmean.y += (Pm[4] * m_w - Pm[7] * mul1) * m2x + (Pm[5] * m_w - Pm[7] * mul2) * m2y;
    dmean.z += (Pm[8] * m_w - Pm[11] * mul1) * m2x + (Pm[9] * m_w - Pm[11] * mul2) * m2y;

    // ---- SH colour backward (CR/backward.cu:12-146), the clamp mask zeroing its channels (:26-28)
    if (do_sh) {
        const float3 v = make_float3(mean.x - c.campos[0], mean.y - c.campos[1], mean.z - c.campos[2]);
        const float3 g = make_float3((cm & 1) ? 0.f : dcol.x, (cm & 2) ? 0.f : dcol.y, (cm & 4) ? 0.f : dcol.z);
        if constexpr (SHM == kShNow)
            sh_dir_backward(sh, D, M, v, g, dmean);
        else
            out.sh_defer(v, g);
    }
    out.dmean(dmean);

    // ---- scale / rotation backward (CR/backward.cu:296-365, called when scales are given, :427-428)
    if (gi.have_scales) {
        const float r_ = q.x, x = q.y, y = q.z, z = q.w;
        // Rg[col][row] = the reference's GLM rotation (R_std transposed)
        const float Rg[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r_ * z), 2.f * (x * z + r_ * y)},
                                {2.f * (x * y + r_ * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r_ * x)},
                                {2.f * (x * z - r_ * y), 2.f * (y * z + r_ * x), 1.f - 2.f * (x * x + y * y)}};
        const float s[3] = {gi.scale_modifier * sc3.x, gi.scale_modifier * sc3.y, gi.scale_modifier * sc3.z};
        const float dS[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                                {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                                {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
        // dMt[r][c] = dL_dM[c][r], dL_dM = 2 M dSigma (GLM product), M[k][r] = s_r Rg[k][r]
        float dMt[3][3];
        for (int c = 0; c < 3; c++)
            for (int rr = 0; rr < 3; rr++)
                dMt[rr][c] = 2.f * s[rr] * (Rg[0][rr] * dS[c][0] + Rg[1][rr] * dS[c][1] + Rg[2][rr] * dS[c][2]);
        // dot(Rt[i], dL_dMt[i]) -- the reference leaves the scale modifier out here
        const float ds0 = Rg[0][0] * dMt[0][0] + Rg[1][0] * dMt[0][1] + Rg[2][0] * dMt[0][2];
        const float ds1 = Rg[0][1] * dMt[1][0] + Rg[1][1] * dMt[1][1] + Rg[2][1] * dMt[1][2];
        const float ds2 = Rg[0][2] * dMt[2][0] + Rg[1][2] * dMt[2][1] + Rg[2][2] * dMt[2][2];
        const float3 dscale = make_float3(ds0, ds1, ds2);
        for (int i = 0; i < 3; i++)
            for (int kk = 0; kk < 3; kk++) dMt[i][kk] *= s[i];
        float4 dq;
        dq.x = 2.f * z * (dMt[0][1] - dMt[1][0]) + 2.f * y * (dMt[2][0] - dMt[0][2]) +
               2.f * x * (dMt[1][2] - dMt[2][1]);
        dq.y = 2.f * y * (dMt[1][0] + dMt[0][1]) + 2.f * z * (dMt[2][0] + dMt[0][2]) +
               2.f * r_ * (dMt[1][2] - dMt[2][1]) - 4.f * x * (dMt[2][2] + dMt[1][1]);
        dq.z = 2.f * x * (dMt[1][0] + dMt[0][1]) + 2.f * r_ * (dMt[2][0] - dMt[0][2]) +
               2.f * z * (dMt[1][2] + dMt[2][1]) - 4.f * y * (dMt[2][2] + dMt[0][0]);
        dq.w = 2.f * r_ * (dMt[0][1] - dMt[1][0]) + 2.f * x * (dMt[2][0] + dMt[0][2]) +
               2.f * y * (dMt[1][2] + dMt[2][1]) - 4.f * z * (dMt[1][1] + dMt[0][0]);
        out.scale_rot(true, dscale, dq);
    } else {
        out.scale_rot(false, make_float3(0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f));
    }
}


// ---- 3. fused per-Gaussian backward ---------------------------------------------
// (Folding the record sums into this kernel was measured slower: the sums' dependent loads
// then run at this kernel's LDS-limited occupancy.)
// The SH rows go through LDS 32 at a time at the end of the kernel (lanes 0-31, then 32-63): 6.6 KiB
// of LDS per wave instead of 13, twice the waves per CU.
constexpr int kGbShRows = 32;
// Live-list entries per gauss_bwd wave (one per lane).
constexpr int kGbListE = 64;
// LIST: lane i of the grid takes entry i of the live list (the Gaussians with a gradient,
// gauss_reduce); the outputs were zero-filled, so no other row is touched.  At
// 1M@1080p that is ~2000 waves instead of 15625.
// The workgroup is one wave: the SH pass's LDS hand-offs need only the wave's own in-order LDS,
// not __syncthreads, whose fence also waits for every store the wave has issued.
__device__ __forceinline__ void gb_sync() {
    wave_lds_sync();
}
// The rows of one wave: Gaussians g0 + lane (dense), or each lane's idx (LIST; a.P: none).  TOUCHED (the
// atomic backward): the sums are the accumulator rows render_bwd added into, read and zeroed here.
constexpr int kGbShFloats = kGbShRows * kShStride;  // one wave's SH staging (LDS)
template <int SH_MODE, bool LIST, bool TOUCHED>
__device__ __forceinline__ void gauss_bwd_rows(const GaussBwdArgs& a, const int g0, const int idx, float* s_sh) {
    const int lane = threadIdx.x & 63;
    const int nvalid = min(64, a.P - g0);
    const int M = a.M;

    const ShAddr sh_src{a.shs, a.dc, M};
    const ShGradAddr sh_dst{a.dL_dsh, a.dL_ddc, M};
    constexpr bool kShLate = SH_MODE != kShGlobal;  // the SH backward deferred to the LDS pass at the end
    // deferred SH backward (kShLate): its inputs, and the 3-D mean gradient it adds to
    bool sh_late = false;
    float3 sh_v = make_float3(0.f, 0.f, 0.f), sh_g = sh_v, dmean_late = sh_v;

    const bool valid = idx < a.P;
    // The summed render gradients decide everything below: a Gaussian whose ten sums are all
    // zero -- culled, or visible but behind saturated pixels everywhere (about 86% of a 1M@1080p
    // frame) -- has all-zero parameter gradients, so it only writes zeros: none of its geometry
    // and none of its 192-byte SH row is read.
    float4 sa = make_float4(0.f, 0.f, 0.f, 0.f), sb = sa;
    float2 sc = make_float2(0.f, 0.f);
    int rad = 0;
    if (valid) {
        rad = a.radii[idx];
        if constexpr (TOUCHED) {
            const float4* row = a.acc + (size_t)idx * kAccRow4;
            sa = row[0];
            sb = row[1];
            const float4 c4 = row[2];
            sc = make_float2(c4.x, c4.y);
        } else {  // (record path: gauss_reduce's per-Gaussian sums)
            sa = a.sums.a[idx];
            sb = a.sums.b[idx];
            sc = a.sums.c[idx];
        }
    }
    const bool any_grad = (sa.x != 0.f) | (sa.y != 0.f) | (sa.z != 0.f) | (sa.w != 0.f) | (sb.x != 0.f) |
                          (sb.y != 0.f) | (sb.z != 0.f) | (sb.w != 0.f) | (sc.x != 0.f) | (sc.y != 0.f);
    if constexpr (TOUCHED) {  // the row back to zero for the next backward of the same forward (its sums are read)
        if (valid) {
            float4* row = a.acc + (size_t)idx * kAccRow4;
            row[0] = row[1] = row[2] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    const bool visible = valid && rad > 0 && any_grad;
    if (valid && !visible) {
        if (!a.sparse) {  // (sparse: the outputs were zero-filled beforehand)
            store3(a.dL_dmean2D, idx, 0.f, 0.f, 0.f);
            if (a.dL_dconic) reinterpret_cast<float4*>(a.dL_dconic)[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
            a.dL_dopacity[idx] = 0.f;
            store3(a.dL_dcolor, idx, 0.f, 0.f, 0.f);
            if (a.dL_dinvdepth) a.dL_dinvdepth[idx] = 0.f;
            store3(a.dL_dmean3D, idx, 0.f, 0.f, 0.f);
            for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = 0.f;
            if (a.dL_dscale) store3(a.dL_dscale, idx, 0.f, 0.f, 0.f);
            if (a.dL_drot) reinterpret_cast<float4*>(a.dL_drot)[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (a.dL_dsh || a.dL_ddc) {
            if constexpr (kShLate) {
                // rows zeroed in the SH pass below
            } else if (!a.sparse) {
                const ShGlobal acc{sh_src, sh_dst, idx};
                for (int k = 0; k < M; k++) acc.store(k, make_float3(0.f, 0.f, 0.f));
            }
        }
    }
    if (visible) {
        // ---- summed render gradients of this Gaussian (loaded above): colour, inverse depth,
        // mean2D, opacity, and dL/dconic in the reference's convention (CR/backward.cu:604-606)
        store3(a.dL_dmean2D, idx, sb.x, sb.y, 0.f);
        store3(a.dL_dcolor, idx, sa.x, sa.y, sa.z);
        if (a.dL_dconic) reinterpret_cast<float4*>(a.dL_dconic)[idx] = make_float4(sc.x, sb.w, 0.f, sc.y);
        if (a.dL_dinvdepth) a.dL_dinvdepth[idx] = sa.w;

        // ---- computeCov2DCUDA, the mean chain, SH and scale/rotation (view_backward, one view)
        const ViewCam cam{a.viewmatrix, a.projmatrix, a.campos, a.tan_fovx, a.tan_fovy,
                          a.focal_x,    a.focal_y,    a.antialiasing, a.have_invdepth};
        GaussIn gi;
        gi.have_scales = a.scales != nullptr;
        gi.mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
        gi.sc3 = make_float3(0.f, 0.f, 0.f);
        gi.q = make_float4(1.f, 0.f, 0.f, 0.f);
        if (a.scales) {
            gi.sc3 = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
            gi.q = reinterpret_cast<const float4*>(a.rotations)[idx];
        }
        gi.cov3D = a.cov3D_precomp ? a.cov3D_precomp + 6 * idx : nullptr;
        gi.scale_modifier = a.scale_modifier;
        gi.opacity = a.opacities + idx;
        // outputs stored as they are formed; dL/dmean3D waits for a deferred SH pass
        struct Sink {
            const GaussBwdArgs& a;
            int idx;
            bool& sh_late;
            float3 &sh_v, &sh_g, &dmean_late;
            __device__ __forceinline__ void dop(float v) const { a.dL_dopacity[idx] = v; }
            __device__ __forceinline__ void dcov(const float (&d)[6]) const {
                for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = d[k];
            }
            __device__ __forceinline__ void sh_defer(float3 v, float3 g) const {
                sh_late = true;
                sh_v = v;
                sh_g = g;
            }
            // kept in a register and stored by the caller (after the SH pass adds the direction term, when
            // there is one): choosing here between the global store and the local made the compiler select
            // between a global and a private address, and dmean_late lived in scratch memory
            __device__ __forceinline__ void dmean(float3 m) const { dmean_late = m; }
            __device__ __forceinline__ void scale_rot(bool have, float3 ds, float4 dq) const {
                if (have || a.dL_dscale) store3(a.dL_dscale, idx, ds.x, ds.y, ds.z);
                if (have || a.dL_drot) reinterpret_cast<float4*>(a.dL_drot)[idx] = dq;
            }
        } sink{a, idx, sh_late, sh_v, sh_g, dmean_late};
        const bool do_sh = a.shs || a.dc;
        const uint8_t cm = do_sh ? a.geom.clamped[idx] : 0;
        if constexpr (kShLate)
            view_backward<kShDefer>(cam, gi, sa, sb, sc, cm, do_sh, a.D, M, ShLds{nullptr}, sink);
        else
            view_backward<kShNow>(cam, gi, sa, sb, sc, cm, do_sh, a.D, M, ShGlobal{sh_src, sh_dst, idx}, sink);
        if (!sh_late) store3(a.dL_dmean3D, idx, dmean_late.x, dmean_late.y, dmean_late.z);
        if (!do_sh && (a.dL_dsh || a.dL_ddc)) {  // colours precomputed: dL/dSH is zero
            const ShGlobal acc{sh_src, sh_dst, idx};
            for (int k = 0; k < M; k++) acc.store(k, make_float3(0.f, 0.f, 0.f));
        }
    }

    if constexpr (kShLate) {
        // SH backward, half a wave at a time through LDS: coalesced stage-in of 32 rows,
        // their lanes evaluate it in place, coalesced write-back of the 32 dL/dSH rows
        const unsigned long long need = __ballot(sh_late);  // rows whose SH is read at all
        for (int half = 0; half < 2; half++) {
            const int rows = LIST ? kGbShRows : min(kGbShRows, nvalid - half * kGbShRows);
            if (rows <= 0) break;  // wave-uniform
            if constexpr (LIST)  // the lanes' rows, wherever they are
                sh_gather_in<kGbShRows, 64, SH_MODE == kShLdsSplit>(sh_src, sh_late ? idx : -1, half * kGbShRows, s_sh,
                                                                   kShStride, lane);
            else
                sh_stage_in<kGbShRows, 64, SH_MODE == kShLdsSplit>(sh_src, g0 + half * kGbShRows, rows, s_sh,
                                                                  kShStride, lane, need >> (half * kGbShRows));
            gb_sync();
            if ((lane >> 5) == half && idx < a.P) {
                float* row = &s_sh[(lane & 31) * kShStride];
                if (sh_late) {
                    // split layout: pin the view vector here -- otherwise the compiler evaluates the SH
                    // basis ahead of the row gather and the barrier, and the values held across it push
                    // the list kernel to 1-3 waves per SIMD.  (The pin moves no arithmetic: with SLP
                    // vectorisation off and contraction per expression, build.py, both layouts round
                    // alike -- test_separate_sh.)
                    float3 v = sh_v;
                    if constexpr (SH_MODE == kShLdsSplit)
                        asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z));
                    float3 dm = dmean_late;
                    sh_dir_backward(ShLds{row}, a.D, M, v, sh_g, dm);
                    store3(a.dL_dmean3D, idx, dm.x, dm.y, dm.z);
                } else if (!a.sparse || SH_MODE == kShLdsSplit) {  // split: see sh_stage_out
                    for (int k = 0; k < kShRowF; k += 4)
                        *reinterpret_cast<float4*>(&row[k]) = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            gb_sync();
            if constexpr (LIST) {
                if (a.dL_dsh || a.dL_ddc)
                    sh_gather_out<kGbShRows, 64, SH_MODE == kShLdsSplit>(sh_dst, sh_late ? idx : -1, half * kGbShRows,
                                                                        s_sh, kShStride, lane);
            } else if (a.dL_dsh || a.dL_ddc) {
                sh_stage_out<kGbShRows, 64, SH_MODE == kShLdsSplit>(sh_dst, g0 + half * kGbShRows, rows, s_sh,
                                                                   kShStride, lane,
                                                                   a.sparse ? need >> (half * kGbShRows) : ~0ull);
            }
            gb_sync();
        }
    }
}

// The live-list grid is sized for the worst case (every Gaussian listed: 64 shards x live_cap / E blocks, 15.7k
// at 1M@1080p, 78k at 5M@4K) while ~2000 blocks have entries; every surplus block is a wave launched to read a
// counter and exit (a grid-strided walk over the virtual blocks measured no better).
template <int SH_MODE, bool LIST = false>
__global__ void __launch_bounds__(64) gauss_bwd_kernel(GaussBwdArgs a) {
    __shared__ __attribute__((aligned(16))) float s_sh[SH_MODE != kShGlobal ? kGbShFloats : 4];
    const int lane = threadIdx.x;
    const uint32_t blk = blockIdx.x;
    if constexpr (LIST) {  // block b: entries [E (b / shards), +E) of shard b % shards, E = kGbListE
        const uint32_t shard = blk % kLiveShards, k0 = (blk / kLiveShards) * kGbListE;
        const uint32_t n = a.live_count[shard * kLiveCntStride];
        if (k0 >= n) return;  // uniform: past the shard's list (the grid is sized for the worst case)
        const int idx = lane < kGbListE && k0 + lane < n ? (int)a.live[(size_t)shard * a.live_cap + k0 + lane] : a.P;
        gauss_bwd_rows<SH_MODE, true, false>(a, (int)blk * 64, idx, s_sh);
    } else {
        gauss_bwd_rows<SH_MODE, false, false>(a, (int)blk * 64, (int)blk * 64 + lane, s_sh);
    }
}

// The atomic backward's per-Gaussian pass (bwd_atomic): a workgroup of kTouchedWaves waves per run of
// consecutive Gaussians reads the run's touched bits (render_bwd set them; cleared as read), lists the touched
// Gaussians in LDS, and wave w runs the live-list backward over list entries [64 w, 64 w + 64) -- the waves
// past the list skip -- with the sums read from, and the rows then zeroed in, the accumulator.  One kernel
// where a gauss_live pass listed the Gaussians into shards and moved their sums to list order for the list
// kernel (1M@1080p -6.8 us per step, 500k -9.3, r7e).  Two waves per workgroup: at 1M@1080p a run of 128
// holds ~17 touched Gaussians, so one wave works while the workgroup holds the LDS of its waves -- against
// four waves per run of 256, gauss_bwd -1.8 / -2.0 us at 1M (r7r, r7s), equal at 500k; one wave per run of
// 64: +6.5 us.
//   RUNS = false: runs of 128, one list of at most 128, no loop (the 1080p frames: ~13% of a 1M view touched).
//   RUNS = true: runs of 128 << touched_shift, sub-run by sub-run of 128 appended to a ring list and flushed
// 128 at a time (and the rest at the end), so the waves stay full where few Gaussians are touched: 5M@4K
// gauss_bwd 120 -> 56 us with runs of 2048 (r7g; 49 us with two waves, r7s).  The loop around the row
// backward costs registers (153 -> 197 VGPRs, combined SH layout) and 3-5 us at 1080p, hence two forms
// ("touched_run", api.hip).
constexpr int kTouchedWaves = 2;
constexpr int kTouchedSub = 64 * kTouchedWaves;  // Gaussians per sub-run (one bit per thread)
constexpr uint32_t kTouchedShiftMax = 5;         // at most 32 sub-runs per workgroup: a touched word per thread
constexpr uint32_t kTouchedRing = 2 * kTouchedSub;
static_assert((kTouchedSub << kTouchedShiftMax) / 32 == kTouchedSub, "one touched word per thread at most");
template <int SH_MODE, bool RUNS>
__global__ void __launch_bounds__(64 * kTouchedWaves) gauss_bwd_touched_kernel(GaussBwdArgs a) {
    __shared__ __attribute__((aligned(16))) float s_sh[kTouchedWaves][SH_MODE != kShGlobal ? kGbShFloats : 4];
    __shared__ uint32_t s_list[RUNS ? kTouchedRing : kTouchedSub];
    __shared__ uint32_t s_words[RUNS ? kTouchedSub : 1];
    __shared__ uint32_t s_cnt[kTouchedWaves];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if constexpr (!RUNS) {
        const uint32_t g = blockIdx.x * (uint32_t)kTouchedSub + threadIdx.x;
        const uint32_t w = g < (uint32_t)a.P ? a.touched[g >> 5] : 0u;  // (each word read by 32 lanes)
        const unsigned long long m = __ballot((w >> (lane & 31)) & 1u);
        if (lane == 0) s_cnt[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t base = 0, total = 0;
#pragma unroll
        for (int k = 0; k < kTouchedWaves; k++) {
            const uint32_t c = s_cnt[k];
            base += k < wave ? c : 0u;
            total += c;
        }
        if ((m >> lane) & 1ull) s_list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = g;
        if ((lane & 31) == 0 && w) a.touched[g >> 5] = 0u;  // (after the ballot read it)
        __syncthreads();
        const uint32_t k0 = 64u * (uint32_t)wave;
        if (k0 >= total) return;  // uniform per wave
        const int idx = k0 + (uint32_t)lane < total ? (int)s_list[k0 + lane] : a.P;
        gauss_bwd_rows<SH_MODE, true, true>(a, 0, idx, s_sh[wave]);
    } else {
        const int nsub = 1 << a.touched_shift;
        const uint32_t run0 = blockIdx.x * ((uint32_t)kTouchedSub << a.touched_shift);
        {
            const uint32_t nwords = (uint32_t)(kTouchedSub / 32) << a.touched_shift;
            const uint32_t wi = (run0 >> 5) + threadIdx.x;
            uint32_t w = 0;
            if (threadIdx.x < nwords && wi < ((uint32_t)a.P + 31u) >> 5) {
                w = a.touched[wi];
                if (w) a.touched[wi] = 0u;  // restored for the next backward of the same forward
            }
            s_words[threadIdx.x] = w;
        }
        __syncthreads();
        uint32_t head = 0, tail = 0;  // the ring's listed entries [head, tail) (uniform)
        for (int j = 0; j < nsub; j++) {
            const uint32_t g = run0 + (uint32_t)(j * kTouchedSub) + threadIdx.x;
            const uint32_t w = s_words[j * (kTouchedSub / 32) + (threadIdx.x >> 5)];
            const unsigned long long m = __ballot((w >> (lane & 31)) & 1u);
            if (lane == 0) s_cnt[wave] = (uint32_t)__popcll(m);
            __syncthreads();  // (also: every wave's reads of the ring's last flush are done)
            uint32_t base = 0, total = 0;
#pragma unroll
            for (int k = 0; k < kTouchedWaves; k++) {
                const uint32_t c = s_cnt[k];
                base += k < wave ? c : 0u;
                total += c;
            }
            if ((m >> lane) & 1ull)
                s_list[(tail + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))) % kTouchedRing] = g;
            tail += total;
            __syncthreads();
            // flush: 256 at a time, and at the last sub-run the rest (tail - head < 2 x 256 here)
            while (tail - head >= (uint32_t)kTouchedSub || (j == nsub - 1 && tail > head)) {  // uniform
                const uint32_t n = min(tail - head, (uint32_t)kTouchedSub);
                const uint32_t k0 = 64u * (uint32_t)wave;
                if (k0 < n) {  // uniform per wave
                    const int idx = k0 + (uint32_t)lane < n ? (int)s_list[(head + k0 + lane) % kTouchedRing] : a.P;
                    gauss_bwd_rows<SH_MODE, true, true>(a, 0, idx, s_sh[wave]);
                }
                head += n;
            }
        }
    }
}

// ---- 4. the same backward over several views' summed render gradients -----------
// Multi-GPU (distributed.py ViewExchange): every rank all-gathers the
// other ranks' per-Gaussian render-gradient sums (a "view block": camera header, 10 floats
// and a flag word per Gaussian, kViewBlock* in gsr_common.h) instead of all-reducing the
// 59-float parameter gradients, and runs this kernel once: one lane per Gaussian loops over
// the views, evaluates view_backward for each view in which the Gaussian is visible, and
// sums the parameter gradients in registers.  Every rank runs it on the same gathered bytes,
// so the replicas' gradients are bitwise identical.
// Phase 1 reads the staged (or global) SH rows for the view-direction gradient and drops
// the per-coefficient products; phase 2 forms dL/dSH_k = sum over views of B_k(dir_v) g_v
// one SH band at a time (bands are compile-time, so the band's accumulators stay in
// registers), recomputing dir_v and g_v from the view blocks -- dL/dSH does not depend on
// the SH values, so the 48 accumulators of all coefficients are never live at once.
template <bool LDS>
struct ShReadOnly {
    const float* lds_row;  // staged row (LDS variants)
    ShAddr src;            // global rows otherwise
    int idx;
    __device__ __forceinline__ float3 load(int k) const {
        if constexpr (LDS) return make_float3(lds_row[3 * k], lds_row[3 * k + 1], lds_row[3 * k + 2]);
        const float* c = src.coef(idx, k);
        return make_float3(c[0], c[1], c[2]);
    }
    __device__ __forceinline__ void store(int, float3) const {}
};
// A view's flag word and summed render gradients for Gaussian idx: from a dense view block, or
// (packed mode, a.flags set) the flag array and the packed entry it indexes (entry layout:
// index bits, a.xyz | a.w, b.xyz | b.w, c.xy, flag bits -- view_pack_scatter_kernel).
template <bool PACKED>
__device__ __forceinline__ uint32_t view_flag(const ViewsBwdArgs& a, const float* blk, int v, int idx) {
    if constexpr (PACKED) return a.flags[(size_t)v * a.P + idx];
    return reinterpret_cast<const uint32_t*>(blk + kViewBlockHeader + 10 * (size_t)a.P)[idx];
}
template <bool PACKED>
__device__ __forceinline__ void view_sums(const ViewsBwdArgs& a, const float* blk, uint32_t flags, int idx,
                                          float4& sa, float4& sb, float2& sc) {
    if constexpr (PACKED) {
        const float4* e = reinterpret_cast<const float4*>(blk + kViewBlockHeader + (size_t)kViewPackEntry * (flags >> 4));
        const float4 e0 = e[0], e1 = e[1], e2 = e[2];
        sa = make_float4(e0.y, e0.z, e0.w, e1.x);
        sb = make_float4(e1.y, e1.z, e1.w, e2.x);
        sc = make_float2(e2.y, e2.z);
    } else {
        const float* sums = blk + kViewBlockHeader;
        sa = reinterpret_cast<const float4*>(sums)[idx];
        sb = reinterpret_cast<const float4*>(sums + 4 * (size_t)a.P)[idx];
        sc = reinterpret_cast<const float2*>(sums + 8 * (size_t)a.P)[idx];
    }
}
template <bool PACKED>
__device__ __forceinline__ float4 view_sums_a(const ViewsBwdArgs& a, const float* blk, uint32_t flags, int idx) {
    if constexpr (PACKED) {
        const float4* e = reinterpret_cast<const float4*>(blk + kViewBlockHeader + (size_t)kViewPackEntry * (flags >> 4));
        const float4 e0 = e[0], e1 = e[1];
        return make_float4(e0.y, e0.z, e0.w, e1.x);
    }
    return reinterpret_cast<const float4*>(blk + kViewBlockHeader)[idx];
}

template <int K0, int K1>
struct ShBand {  // accumulates B_k g for K0 <= k < K1; SH values are not needed (read as 0)
    float* acc;
    __device__ __forceinline__ float3 load(int) const { return make_float3(0.f, 0.f, 0.f); }
    __device__ __forceinline__ void store(int k, float3 v) const {
        if (k >= K0 && k < K1) {
            acc[3 * (k - K0)] += v.x;
            acc[3 * (k - K0) + 1] += v.y;
            acc[3 * (k - K0) + 2] += v.z;
        }
    }
};

// dL/dSH of band [K0, K1) for lane idx, summed over the views it is visible in; written to
// the lane's LDS row (LDS variants) or straight to global memory
template <int K0, int K1, int SH_MODE, bool PACKED>
__device__ __forceinline__ void views_sh_band(const ViewsBwdArgs& a, int idx, float3 mean, float* row,
                                              const ShGradAddr& dst) {
    float acc[3 * (K1 - K0)];
#pragma unroll
    for (int i = 0; i < 3 * (K1 - K0); i++) acc[i] = 0.f;
#pragma unroll 1
    for (int v = 0; v < a.n_views; v++) {
        const float* blk = a.blocks + (size_t)v * a.block_floats;
        const uint32_t flags = view_flag<PACKED>(a, blk, v, idx);
        if (!(flags & 1u)) continue;
        const float* cp = blk + kViewCamPos;
        const float3 d = make_float3(mean.x - cp[0], mean.y - cp[1], mean.z - cp[2]);
        const float len = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        const float4 sa = view_sums_a<PACKED>(a, blk, flags, idx);
        const float3 g = make_float3((flags & 2u) ? 0.f : sa.x, (flags & 4u) ? 0.f : sa.y, (flags & 8u) ? 0.f : sa.z);
        float ddx, ddy, ddz;
        sh_backward(ShBand<K0, K1>{acc}, a.D, a.M, d.x / len, d.y / len, d.z / len, g, ddx, ddy, ddz);
    }
#pragma unroll
    for (int k = K0; k < K1; k++) {
        const float x = acc[3 * (k - K0)], y = acc[3 * (k - K0) + 1], z = acc[3 * (k - K0) + 2];
        if constexpr (SH_MODE != kShGlobal) {
            row[3 * k] = x;
            row[3 * k + 1] = y;
            row[3 * k + 2] = z;
        } else if (k < a.M) {
            float* c = dst.coef(idx, k);
            c[0] = x;
            c[1] = y;
            c[2] = z;
        }
    }
}

// 3 waves per SIMD (the LDS limit of the SH staging): the register allocator then spills a
// few values but the per-view latency chains overlap better (8 views: 0.50 -> 0.44 ms, r1af)
template <int SH_MODE, bool PACKED, bool LIST = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3, 3))) gauss_bwd_views_kernel(ViewsBwdArgs a) {
    __shared__ __attribute__((aligned(16))) float s_sh[SH_MODE != kShGlobal ? 64 * kShStride : 4];
    const int lane = threadIdx.x;
    const int g0 = blockIdx.x * 64;
    int idx = g0 + lane;
    if constexpr (LIST) {  // a lane per Gaussian some view flags (the outputs were zeroed beforehand)
        const uint32_t shard = blockIdx.x % kLiveShards, k0 = (blockIdx.x / kLiveShards) * 64;
        const uint32_t n = a.live_count[shard * kLiveCntStride];
        if (k0 >= n) return;  // uniform: past the shard's list
        idx = k0 + lane < n ? (int)a.live[(size_t)shard * a.live_cap + k0 + lane] : a.P;
    }
    const int nvalid = min(64, a.P - g0);
    const int M = a.M;
    const ShAddr sh_src{a.shs, a.dc, M};
    const ShGradAddr sh_dst{a.dL_dsh, a.dL_ddc, M};
    if constexpr (SH_MODE != kShGlobal) {
        if constexpr (LIST)
            sh_gather_in<64, 64, SH_MODE == kShLdsSplit>(sh_src, idx < a.P ? idx : -1, 0, s_sh, kShStride, lane);
        else
            sh_stage_in<64, 64, SH_MODE == kShLdsSplit>(sh_src, g0, nvalid, s_sh, kShStride, lane);
        __syncthreads();
    }
    const bool valid = idx < a.P;
    float3 mean = make_float3(0.f, 0.f, 0.f);
    // ---- phase 1: geometry gradients, summed over views
    if (valid) {
        GaussIn gi;
        gi.mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
        mean = gi.mean;
        gi.have_scales = true;
        gi.sc3 = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
        gi.q = reinterpret_cast<const float4*>(a.rotations)[idx];
        gi.cov3D = nullptr;
        gi.scale_modifier = a.scale_modifier;
        gi.opacity = a.opacities + idx;
        const ShReadOnly<SH_MODE != kShGlobal> shr{SH_MODE != kShGlobal ? &s_sh[lane * kShStride] : nullptr, sh_src,
                                                   idx};
        // the parameter gradients summed over the views (dL/dcov3D is not an output here)
        struct Sink {
            float3 dmean_sum = make_float3(0.f, 0.f, 0.f), dscale_sum = make_float3(0.f, 0.f, 0.f);
            float4 drot_sum = make_float4(0.f, 0.f, 0.f, 0.f);
            float dop_sum = 0.f;
            __device__ __forceinline__ void dop(float v) { dop_sum += v; }
            __device__ __forceinline__ void dcov(const float (&)[6]) {}
            __device__ __forceinline__ void sh_defer(float3, float3) {}
            __device__ __forceinline__ void dmean(float3 m) {
                dmean_sum.x += m.x; dmean_sum.y += m.y; dmean_sum.z += m.z;
            }
            __device__ __forceinline__ void scale_rot(bool, float3 ds, float4 dq) {
                dscale_sum.x += ds.x; dscale_sum.y += ds.y; dscale_sum.z += ds.z;
                drot_sum.x += dq.x; drot_sum.y += dq.y; drot_sum.z += dq.z; drot_sum.w += dq.w;
            }
        } sink;
        uint32_t flags_next = a.n_views > 0 ? view_flag<PACKED>(a, a.blocks, 0, idx) : 0u;
#pragma unroll 1
        for (int v = 0; v < a.n_views; v++) {
            const float* blk = a.blocks + (size_t)v * a.block_floats;
            const uint32_t flags = flags_next;
            if (v + 1 < a.n_views) flags_next = view_flag<PACKED>(a, blk + a.block_floats, v + 1, idx);
            if (!(flags & 1u)) continue;  // not visible in view v: no gradient from it
            const ViewCam cam{blk + kViewCamView, blk + kViewCamProj, blk + kViewCamPos, blk[kViewCamTanX],
                              blk[kViewCamTanY],  blk[kViewCamFocalX], blk[kViewCamFocalY],
                              (int)__float_as_uint(blk[kViewCamAA]), (int)__float_as_uint(blk[kViewCamInvDepth])};
            float4 sa, sb;
            float2 sc;
            view_sums<PACKED>(a, blk, flags, idx, sa, sb, sc);
            view_backward<kShNow>(cam, gi, sa, sb, sc, (uint8_t)((flags >> 1) & 7u), true, a.D, M, shr, sink);
        }
        store3(a.dL_dmean3D, idx, sink.dmean_sum.x, sink.dmean_sum.y, sink.dmean_sum.z);
        a.dL_dopacity[idx] = sink.dop_sum;
        store3(a.dL_dscale, idx, sink.dscale_sum.x, sink.dscale_sum.y, sink.dscale_sum.z);
        reinterpret_cast<float4*>(a.dL_drot)[idx] = sink.drot_sum;
    }
    // ---- phase 2: dL/dSH band by band (CR/backward.cu:43-127 products, summed over views)
    if constexpr (SH_MODE != kShGlobal) __syncthreads();  // the staged SH rows are read for the last time
    float* row = SH_MODE != kShGlobal ? &s_sh[lane * kShStride] : nullptr;
    if (valid) {
        // one walk over the views for every band: phase 1's registers are dead here, so the 48
        // accumulators fit under its peak (four walks -- one per band -- cost 0.12 of 0.28 ms at 8
        // views, r3z)
        if (a.D > 2) views_sh_band<0, 16, SH_MODE, PACKED>(a, idx, mean, row, sh_dst);
        else if (a.D > 1) views_sh_band<0, 9, SH_MODE, PACKED>(a, idx, mean, row, sh_dst);
        else if (a.D > 0) views_sh_band<0, 4, SH_MODE, PACKED>(a, idx, mean, row, sh_dst);
        else views_sh_band<0, 1, SH_MODE, PACKED>(a, idx, mean, row, sh_dst);
        const int K = (a.D + 1) * (a.D + 1);
        if constexpr (SH_MODE != kShGlobal) {
            for (int k = K; k < 16; k++) row[3 * k] = row[3 * k + 1] = row[3 * k + 2] = 0.f;
        } else {
            for (int k = K; k < M; k++) {
                float* c = sh_dst.coef(idx, k);
                c[0] = c[1] = c[2] = 0.f;
            }
        }
    }
    if constexpr (SH_MODE != kShGlobal) {
        __syncthreads();
        if constexpr (LIST)
            sh_gather_out<64, 64, SH_MODE == kShLdsSplit>(sh_dst, idx < a.P ? idx : -1, 0, s_sh, kShStride, lane);
        else
            sh_stage_out<64, 64, SH_MODE == kShLdsSplit>(sh_dst, g0, nvalid, s_sh, kShStride, lane);
    }
}

hipError_t launch_gauss_bwd_views(const ViewsBwdArgs& a, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    const dim3 grid((a.P + 63) / 64), block(64);
    const bool lds = a.shs && a.dL_dsh && a.M == 16 && (!a.dc || a.dL_ddc) &&
                     ((reinterpret_cast<uintptr_t>(a.shs) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(a.dL_dsh) & 15) == 0);
    if (a.flags && a.live) {  // packed blocks, a lane per Gaussian some view flags (outputs pre-zeroed)
        const dim3 lgrid(kLiveShards * ((a.live_cap + 63) / 64));
        if (lds && a.dc)
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsSplit, true, true>), lgrid, block, 0, stream, a);
        else if (lds)
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsCombined, true, true>), lgrid, block, 0, stream, a);
        else
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShGlobal, true, true>), lgrid, block, 0, stream, a);
    } else if (a.flags) {  // packed blocks (gsr_view_block_index)
        if (lds && a.dc)
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsSplit, true>), grid, block, 0, stream, a);
        else if (lds)
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsCombined, true>), grid, block, 0, stream, a);
        else
            hipLaunchKernelGGL((gauss_bwd_views_kernel<kShGlobal, true>), grid, block, 0, stream, a);
    } else if (lds && a.dc) {
        hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsSplit, false>), grid, block, 0, stream, a);
    } else if (lds) {
        hipLaunchKernelGGL((gauss_bwd_views_kernel<kShLdsCombined, false>), grid, block, 0, stream, a);
    } else {
        hipLaunchKernelGGL((gauss_bwd_views_kernel<kShGlobal, false>), grid, block, 0, stream, a);
    }
    return hipGetLastError();
}

// The header of a view block: the camera, as gauss_bwd_views_kernel reads it.
__global__ void view_header_kernel(float* blk, const float* view, const float* proj, const float* campos,
                                   float tan_fovx, float tan_fovy, float focal_x, float focal_y, int antialiasing,
                                   int have_invdepth) {
    const int t = threadIdx.x;
    if (t < 16) blk[kViewCamView + t] = view[t];
    else if (t < 32) blk[kViewCamProj + t - 16] = proj[t - 16];
    else if (t < 35) blk[kViewCamPos + t - 32] = campos[t - 32];
    else if (t == 35) {
        blk[kViewCamTanX] = tan_fovx;
        blk[kViewCamTanY] = tan_fovy;
        blk[kViewCamFocalX] = focal_x;
        blk[kViewCamFocalY] = focal_y;
        blk[kViewCamAA] = __uint_as_float((uint32_t)antialiasing);
        blk[kViewCamInvDepth] = __uint_as_float((uint32_t)have_invdepth);
    }
}

// ---- sparse view blocks (multi-GPU exchange) ------------------------------------------
// Only the Gaussians with a non-zero render gradient need to travel: behind saturated pixels
// most have none (about 14% of a 1M@1080p view do).  A packed block is the view block's header
// (64 floats, the entry count in float kViewPackCount) followed by count entries of 12 floats:
// Gaussian index (bits), sums.a (4), sums.b (4), sums.c (2), flag word (bits), in Gaussian
// order (a deterministic compaction: per-workgroup counts, one scan, an in-order scatter).
constexpr int kPackThreads = 256;

__device__ __forceinline__ bool view_entry_live(const float* body, uint32_t P, uint32_t g) {
    const float4 a = reinterpret_cast<const float4*>(body)[g];
    const float4 b = reinterpret_cast<const float4*>(body + 4 * (size_t)P)[g];
    const float2 c = reinterpret_cast<const float2*>(body + 8 * (size_t)P)[g];
    const uint32_t f = __float_as_uint(body[10 * (size_t)P + g]);
    return (f & 1u) && ((a.x != 0.f) | (a.y != 0.f) | (a.z != 0.f) | (a.w != 0.f) | (b.x != 0.f) | (b.y != 0.f) |
                        (b.z != 0.f) | (b.w != 0.f) | (c.x != 0.f) | (c.y != 0.f));
}

// rank of this thread among the live threads of its workgroup, and the workgroup's total
__device__ __forceinline__ uint32_t block_live_rank(bool live, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long m = __ballot(live);
    const uint32_t in_wave = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (int k = 0; k < kPackThreads / 64; k++) {
        before += k < w ? s_w[k] : 0u;
        all += s_w[k];
    }
    *total = all;
    return before + in_wave;
}

// (range forms: only Gaussians [g0, g1) are packed, indexed, listed -- one chunk of a chunked exchange,
// distributed.py ViewExchange(chunks=K); entries keep their absolute Gaussian index)
__global__ void __launch_bounds__(kPackThreads) view_pack_count_kernel(uint32_t P, uint32_t g0, uint32_t g1,
                                                                       const float* __restrict__ block,
                                                                       uint32_t* __restrict__ wg_cnt) {
    __shared__ uint32_t s_w[kPackThreads / 64];
    const uint32_t g = g0 + blockIdx.x * kPackThreads + threadIdx.x;
    const bool live = g < g1 && view_entry_live(block + kViewBlockHeader, P, g);
    uint32_t total = 0;
    block_live_rank(live, s_w, &total);
    if (threadIdx.x == 0) wg_cnt[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the per-workgroup counts (in place), total into the packed header
__global__ void __launch_bounds__(1024) view_pack_scan_kernel(uint32_t nb, uint32_t* __restrict__ wg_cnt,
                                                              float* __restrict__ packed, uint32_t* __restrict__ count) {
    __shared__ uint32_t s_tot[1024 / 64];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nb ? wg_cnt[i] : 0u;
        const uint32_t incl = wave_incl_sum(v);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        if (lane == 63) s_tot[w] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int k = 0; k < (int)(blockDim.x / 64); k++) {
            before += k < w ? s_tot[k] : 0u;
            all += s_tot[k];
        }
        if (i < nb) wg_cnt[i] = carry + before + incl - v;
        carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        packed[kViewPackCount] = __uint_as_float(carry);
        if (count) count[0] = carry;
    }
}

__global__ void __launch_bounds__(kPackThreads) view_pack_scatter_kernel(uint32_t P, uint32_t g0, uint32_t g1,
                                                                         const float* __restrict__ block,
                                                                         const uint32_t* __restrict__ wg_off,
                                                                         float* __restrict__ packed,
                                                                         unsigned long long cap) {
    __shared__ uint32_t s_w[kPackThreads / 64];
    if (blockIdx.x == 0 && threadIdx.x < kViewBlockHeader && threadIdx.x != kViewPackCount)
        packed[threadIdx.x] = block[threadIdx.x];
    const float* body = block + kViewBlockHeader;
    const uint32_t g = g0 + blockIdx.x * kPackThreads + threadIdx.x;
    const bool live = g < g1 && view_entry_live(body, P, g);
    uint32_t total = 0;
    const uint32_t pos = wg_off[blockIdx.x] + block_live_rank(live, s_w, &total);
    if (live && pos < cap) {
        const float4 a = reinterpret_cast<const float4*>(body)[g];
        const float4 b = reinterpret_cast<const float4*>(body + 4 * (size_t)P)[g];
        const float2 c = reinterpret_cast<const float2*>(body + 8 * (size_t)P)[g];
        const float f = body[10 * (size_t)P + g];
        float4* e = reinterpret_cast<float4*>(packed + kViewBlockHeader + (size_t)kViewPackEntry * pos);
        e[0] = make_float4(__uint_as_float(g), a.x, a.y, a.z);
        e[1] = make_float4(a.w, b.x, b.y, b.z);
        e[2] = make_float4(b.w, c.x, c.y, f);
    }
}

hipError_t launch_view_pack(uint32_t P, uint32_t g0, uint32_t g1, const float* block, float* packed,
                            unsigned long long cap, uint32_t* scratch, uint32_t* count, hipStream_t stream) {
    const uint32_t nb = (g1 - g0 + kPackThreads - 1) / kPackThreads;
    if (nb == 0) {  // an empty range: a header with no entries
        hipLaunchKernelGGL(view_pack_scan_kernel, dim3(1), dim3(1024), 0, stream, 0u, scratch, packed, count);
        hipLaunchKernelGGL(view_pack_scatter_kernel, dim3(1), dim3(kPackThreads), 0, stream, P, g0, g0, block, scratch,
                           packed, cap);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(view_pack_count_kernel, dim3(nb), dim3(kPackThreads), 0, stream, P, g0, g1, block, scratch);
    hipLaunchKernelGGL(view_pack_scan_kernel, dim3(1), dim3(1024), 0, stream, nb, scratch, packed, count);
    hipLaunchKernelGGL(view_pack_scatter_kernel, dim3(nb), dim3(kPackThreads), 0, stream, P, g0, g1, block, scratch,
                       packed, cap);
    return hipGetLastError();
}

// The flag words of n_views dense view blocks zeroed: gauss_bwd_views_kernel reads a Gaussian's
// sums only when its flag has the visible bit, so after this and the scatter below the sums of
// the Gaussians left out of a packed block are never read, and need no zeroing (a 40-B-per-
// Gaussian memset per view, 320 MB at 8 views, reduced to 4 B).
__global__ void __launch_bounds__(kPackThreads) view_flags_zero_kernel(uint32_t P, float* __restrict__ blocks,
                                                                       unsigned long long block_floats) {
    uint32_t* f = reinterpret_cast<uint32_t*>(blocks + blockIdx.y * block_floats + kViewBlockHeader + 10 * (size_t)P);
    for (uint32_t g = blockIdx.x * kPackThreads + threadIdx.x; g < P; g += gridDim.x * kPackThreads) f[g] = 0u;
}

// packed [n_views][packed_floats] -> dense view blocks [n_views][view_block_floats(P)], whose
// flag words view_flags_zero_kernel cleared: header copy and one entry per thread.
__global__ void __launch_bounds__(kPackThreads) view_unpack_kernel(uint32_t P, const float* __restrict__ packed,
                                                                   unsigned long long packed_floats,
                                                                   float* __restrict__ blocks,
                                                                   unsigned long long block_floats,
                                                                   unsigned long long cap) {
    const uint32_t v = blockIdx.y;
    const float* pk = packed + v * packed_floats;
    float* blk = blocks + v * block_floats;
    if (blockIdx.x == 0 && threadIdx.x < kViewBlockHeader) blk[threadIdx.x] = threadIdx.x == kViewPackCount ? 0.f
                                                                                                       : pk[threadIdx.x];
    uint32_t n = __float_as_uint(pk[kViewPackCount]);
    n = n < cap ? n : (uint32_t)cap;
    float* body = blk + kViewBlockHeader;
    for (uint32_t i = blockIdx.x * kPackThreads + threadIdx.x; i < n; i += gridDim.x * kPackThreads) {
        const float4* e = reinterpret_cast<const float4*>(pk + kViewBlockHeader + (size_t)kViewPackEntry * i);
        const float4 e0 = e[0], e1 = e[1], e2 = e[2];
        const uint32_t g = __float_as_uint(e0.x);
        if (g >= P) continue;  // never for a block packed by view_pack_scatter_kernel
        reinterpret_cast<float4*>(body)[g] = make_float4(e0.y, e0.z, e0.w, e1.x);
        reinterpret_cast<float4*>(body + 4 * (size_t)P)[g] = make_float4(e1.y, e1.z, e1.w, e2.x);
        reinterpret_cast<float2*>(body + 8 * (size_t)P)[g] = make_float2(e2.y, e2.z);
        body[10 * (size_t)P + g] = e2.w;
    }
}

hipError_t launch_view_unpack(uint32_t P, int n_views, const float* packed, unsigned long long packed_floats,
                              float* blocks, unsigned long long cap, hipStream_t stream) {
    if (n_views <= 0) return hipSuccess;
    const size_t bf = view_block_floats(P);
    const uint32_t gz = (P + kPackThreads - 1) / kPackThreads;
    hipLaunchKernelGGL(view_flags_zero_kernel, dim3(gz < 1024 ? (gz ? gz : 1) : 1024, n_views), dim3(kPackThreads), 0,
                       stream, P, blocks, (unsigned long long)bf);
    const uint32_t gx = (uint32_t)((cap + kPackThreads - 1) / kPackThreads);
    hipLaunchKernelGGL(view_unpack_kernel, dim3(gx < 1024 ? (gx ? gx : 1) : 1024, n_views), dim3(kPackThreads), 0,
                       stream, P, packed, packed_floats, blocks, (unsigned long long)bf, cap);
    return hipGetLastError();
}

// Packed mode of the multi-view backward: instead of rebuilding dense view blocks, each view's
// flag array [P] is cleared and, for every packed entry i, set to i << 4 | its flag bits -- one
// 4-byte store per entry instead of four scattered stores of 44 bytes.
__global__ void __launch_bounds__(kPackThreads) view_index_kernel(uint32_t P, const float* __restrict__ packed,
                                                                  unsigned long long packed_floats,
                                                                  uint32_t* __restrict__ flags,
                                                                  unsigned long long cap) {
    const uint32_t v = blockIdx.y;
    const float* pk = packed + v * packed_floats;
    uint32_t n = __float_as_uint(pk[kViewPackCount]);
    n = n < cap ? n : (uint32_t)cap;
    uint32_t* f = flags + (size_t)v * P;
    for (uint32_t i = blockIdx.x * kPackThreads + threadIdx.x; i < n; i += gridDim.x * kPackThreads) {
        const float* e = pk + kViewBlockHeader + (size_t)kViewPackEntry * i;
        const uint32_t g = __float_as_uint(e[0]);
        if (g < P) f[g] = (i << 4) | (__float_as_uint(e[11]) & 15u);
    }
}

__global__ void __launch_bounds__(kPackThreads) flags_zero_kernel(uint32_t P, uint32_t g0, uint32_t g1,
                                                                  uint32_t* __restrict__ flags) {
    uint32_t* f = flags + (size_t)blockIdx.y * P;
    for (uint32_t g = g0 + blockIdx.x * kPackThreads + threadIdx.x; g < g1; g += gridDim.x * kPackThreads) f[g] = 0u;
}

hipError_t launch_view_index(uint32_t P, uint32_t g0, uint32_t g1, int n_views, const float* packed,
                             unsigned long long packed_floats, uint32_t* flags, unsigned long long cap,
                             hipStream_t stream) {
    if (n_views <= 0) return hipSuccess;
    const uint32_t gz = (g1 - g0 + kPackThreads - 1) / kPackThreads;
    hipLaunchKernelGGL(flags_zero_kernel, dim3(gz < 1024 ? (gz ? gz : 1) : 1024, n_views), dim3(kPackThreads), 0,
                       stream, P, g0, g1, flags);
    const uint32_t gx = (uint32_t)((cap + kPackThreads - 1) / kPackThreads);
    hipLaunchKernelGGL(view_index_kernel, dim3(gx < 1024 ? (gx ? gx : 1) : 1024, n_views), dim3(kPackThreads), 0,
                       stream, P, packed, packed_floats, flags, cap);
    return hipGetLastError();
}

// The Gaussians some view flags (visible with a gradient in a packed block), appended to the
// sharded live list (one atomic per wave, kLiveShards counters the caller zeroed).
__global__ void __launch_bounds__(64) views_live_kernel(uint32_t P, uint32_t g0, uint32_t g1, int n_views,
                                                        const uint32_t* __restrict__ flags,
                                                        uint32_t* __restrict__ live, uint32_t* __restrict__ live_count,
                                                        uint32_t live_cap) {
    const uint32_t g = g0 + blockIdx.x * 64 + threadIdx.x;
    bool lv = false;
    if (g < g1)
        for (int v = 0; v < n_views; v++) lv |= (flags[(size_t)v * P + g] & 1u) != 0;
    const unsigned long long m = __ballot(lv);
    if (!m) return;
    const uint32_t shard = blockIdx.x % kLiveShards;
    uint32_t base = 0;
    if (threadIdx.x == 0) base = atomicAdd(&live_count[shard * kLiveCntStride], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, 0);
    if (lv) live[(size_t)shard * live_cap + base + (uint32_t)__popcll(m & ((1ull << threadIdx.x) - 1ull))] = g;
}

hipError_t launch_views_live(uint32_t P, uint32_t g0, uint32_t g1, int n_views, const uint32_t* flags, uint32_t* live,
                             uint32_t* live_count, hipStream_t stream) {
    const hipError_t e = hipMemsetAsync(live_count, 0, sizeof(uint32_t) * kLiveShards * kLiveCntStride, stream);
    if (e != hipSuccess || g1 <= g0) return e;
    // (a range's blocks are at most P's, so live_list_cap(P) bounds every shard)
    hipLaunchKernelGGL(views_live_kernel, dim3((g1 - g0 + 63) / 64), dim3(64), 0, stream, P, g0, g1, n_views, flags,
                       live, live_count, live_list_cap(P));
    return hipGetLastError();
}

hipError_t launch_view_header(float* blk, const float* view, const float* proj, const float* campos, float tan_fovx,
                              float tan_fovy, float focal_x, float focal_y, int antialiasing, int have_invdepth,
                              hipStream_t stream) {
    hipLaunchKernelGGL(view_header_kernel, dim3(1), dim3(64), 0, stream, blk, view, proj, campos, tan_fovx, tan_fovy,
                       focal_x, focal_y, antialiasing, have_invdepth);
    return hipGetLastError();
}

// 16-byte stores (1 KiB per wave-instruction) over each range's aligned body, dwords for its
// unaligned head and tail.  A small grid (kFillBlocks workgroups of 256): beside render_bwd
// it should take few wave slots and only the HBM bandwidth render_bwd leaves idle.  The body
// stores are non-temporal (`nt`): 236 MB of zeros written through the caches evicted the
// records and pixel state render_bwd and gauss_reduce re-read (r2zv: render_bwd 298 -> 290 us,
// gauss_reduce 67 -> 63, preprocess 75.6 -> 72, step -19 us; 32 / 64 / 96 / 128 workgroups
// within noise once the stores stream, r2zw).
constexpr uint32_t kFillBlocks = 64;
__global__ void __launch_bounds__(256) zero_fill_kernel(FillArgs f) {
    zero_fill_part(f, (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x,
                   (unsigned long long)gridDim.x * blockDim.x);
}

hipError_t launch_zero_fill(const FillArgs& f, hipStream_t stream) {
    if (f.count == 0) return hipSuccess;
    hipLaunchKernelGGL(zero_fill_kernel, dim3(kFillBlocks), dim3(256), 0, stream, f);
    return hipGetLastError();
}

hipError_t launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    const dim3 grid((a.P + 63) / 64), block(64);
    const bool lds_ok = a.shs && a.dL_dsh && a.M == 16 && (!a.dc || a.dL_ddc) &&
                        ((reinterpret_cast<uintptr_t>(a.shs) & 15) == 0) &&
                        ((reinterpret_cast<uintptr_t>(a.dL_dsh) & 15) == 0);
    if (a.touched) {  // the atomic backward: runs of touched Gaussians (outputs zero-filled)
        if (a.touched_shift > kTouchedShiftMax) return hipErrorInvalidValue;
        const size_t run = (size_t)kTouchedSub << a.touched_shift;
        const dim3 tgrid((uint32_t)(((size_t)a.P + run - 1) / run)), tblock(64 * kTouchedWaves);
        const bool runs = a.touched_shift > 0;
        void (*k)(GaussBwdArgs);
        if (lds_ok && a.dc)
            k = runs ? gauss_bwd_touched_kernel<kShLdsSplit, true> : gauss_bwd_touched_kernel<kShLdsSplit, false>;
        else if (lds_ok)
            k = runs ? gauss_bwd_touched_kernel<kShLdsCombined, true> : gauss_bwd_touched_kernel<kShLdsCombined, false>;
        else
            k = runs ? gauss_bwd_touched_kernel<kShGlobal, true> : gauss_bwd_touched_kernel<kShGlobal, false>;
        hipLaunchKernelGGL(k, tgrid, tblock, 0, stream, a);
        return hipGetLastError();
    }
    if (a.live && a.sparse) {  // the live list: kLiveShards x live_cap entries at most
        const uint32_t worst = kLiveShards * ((a.live_cap + kGbListE - 1) / kGbListE);
        const dim3 lgrid(worst);
        if (lds_ok && a.dc)
            hipLaunchKernelGGL((gauss_bwd_kernel<kShLdsSplit, true>), lgrid, block, 0, stream, a);
        else if (lds_ok)
            hipLaunchKernelGGL((gauss_bwd_kernel<kShLdsCombined, true>), lgrid, block, 0, stream, a);
        else
            hipLaunchKernelGGL((gauss_bwd_kernel<kShGlobal, true>), lgrid, block, 0, stream, a);
        return hipGetLastError();
    }
    const bool lds = a.shs && a.dL_dsh && a.M == 16 && (!a.dc || a.dL_ddc) &&
                     ((reinterpret_cast<uintptr_t>(a.shs) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(a.dL_dsh) & 15) == 0);
    if (lds && a.dc)
        hipLaunchKernelGGL(gauss_bwd_kernel<kShLdsSplit>, grid, block, 0, stream, a);
    else if (lds)
        hipLaunchKernelGGL(gauss_bwd_kernel<kShLdsCombined>, grid, block, 0, stream, a);
    else
        hipLaunchKernelGGL(gauss_bwd_kernel<kShGlobal>, grid, block, 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr

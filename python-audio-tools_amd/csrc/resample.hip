// resample.hip — MI355X batch sinc resampler (SURVEY §8(a) rows R1–R3):
// the reference's pcmconverter.Resampler (src/pcmconverter.c:370-495,
// float buffers :533-629) over the vendored libsamplerate 0.1.8 sinc
// converter (src/samplerate/src_sinc.c: sinc_*_vari_process :329-420,
// 478-568, 1039-1128; calc_output_* :277-326, 423-475, 908-1036;
// prepare_data :1135-1213), for a batch of tracks.
//
// Coefficients: the MEDIUM table the reference tree holds (src_coeffs.h,
// tools/gen_src_coeffs.py); the reference's own choice, BEST, needs a table
// the tree lacks, so parity is against the CPU restatement
// oracle/resample_port.c, bit for bit, and unpinned to reference output.
//
// Output frame n of a track sits at input frame c_n + frac_n.  The
// reference advances frac by 1/ratio in fp64 through fmod_one (:552-556), a
// serial recurrence, but its arithmetic is exact in two common cases, where
// every state is a multiple of 2^-53 and nothing rounds:
//   * 1/ratio in [0.5, 1) with an even 53-bit numerator D (44.1k -> 48k):
//     frac_n = (n D mod 2^53) 2^-53, c_n = floor(n D / 2^53);
//   * an integer 1/ratio (192k -> 48k): frac_n = 0, c_n = n / ratio.
// Those tracks need no serial pass at all; any other ratio replays the
// fp64 recurrence in one lane per track (k_rs_positions) first.
//
//   k_rs_positions  lane per "serial" track: (c_n, start filter index) per
//                   output, staged through LDS so the stores are coalesced.
//   k_rs_filter     persistent blocks, the float table in LDS; a block takes
//                   1024 consecutive outputs of one track, stages their
//                   input window in LDS as float (x / 2^(bps-1)), and each
//                   thread runs the left and right half filters of its
//                   output (fp64 accumulation tap by tap in the reference's
//                   order, contraction off), scale, float, then
//                   (int)(f * 2^(bps-1)) clamped -- fb_export_frames.
#include <hip/hip_runtime.h>
#include <type_traits>

#include <algorithm>
#include <numeric>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "src_coeffs.h"

#pragma clang fp contract(off)

namespace {

constexpr int kShift = 12;             // SHIFT_BITS (src_sinc.c:40)
constexpr int kChunk = 1024;           // outputs per block iteration
constexpr int kTable = SRC_MEDIUM_HALF_LEN + 2;

enum { POS_CLOSED_FRAC = 0, POS_CLOSED_INT = 1, POS_TABLE = 2 };

struct RsTrack {
    uint64_t in_base;    // first input sample (interleaved index)
    uint64_t in_frames;
    uint64_t out_base;   // first output sample (interleaved index)
    uint64_t out_frames;
    uint64_t pos_base;   // POS_TABLE: first (c, sfi) entry
    uint64_t D;          // POS_CLOSED_FRAC: 2^53 / ratio; POS_CLOSED_INT: 1/ratio
    double float_increment, scale;
    int32_t increment, mode;
    uint64_t chunk_base; // first work chunk of the track (k_rs_filter)
    uint64_t span;       // k_rs_phase: outputs per task (64 x lspan x rows)
    uint32_t period;     // k_rs_phase: outputs per phase cycle (out_rate / gcd)
    uint32_t lspan;      // k_rs_phase: outputs between a wave's lanes (a multiple of period)
    uint32_t wext;       // k_rs_phase: window frames staged past the task's last centre's taps
    uint32_t cls;        // k_rs_phase: ratio class (its phase tables)
};

struct RsParams {
    uint32_t ch, bps, n_tracks, n_chunks, chunk;
    float inv_q, q;
    int32_t lo, hi;
};

// (c_n, start_filter_index) of output n (see the file comment)
__device__ __forceinline__ void position(const RsTrack &T, const int2 *__restrict__ pos,
                                         uint64_t n, int64_t &c, int32_t &sfi)
{
    if (T.mode == POS_CLOSED_FRAC) {
        const uint64_t lo = n * T.D, hi = __umul64hi(n, T.D);
        c = (int64_t)((hi << 11) | (lo >> 53));
        const uint64_t S = lo & ((1ull << 53) - 1ull);
        const double frac = (double)S * 0x1p-53;
        sfi = (int32_t)__double2int_rn((frac * T.float_increment) * (double)(1 << kShift));
    } else if (T.mode == POS_CLOSED_INT) {
        c = (int64_t)(n * T.D);
        sfi = 0;
    } else {
        const int2 p = pos[T.pos_base + n];
        c = (int64_t)(uint32_t)p.x;
        sfi = p.y;
    }
}

// the serial fp64 recurrence (src_sinc.c:522-556) for tracks without a
// closed form: lane per track, 64 steps staged in LDS per flush
__global__ __launch_bounds__(64) void k_rs_positions(const RsTrack *__restrict__ tr,
                                                     const uint32_t *__restrict__ ids, uint32_t n,
                                                     int2 *__restrict__ pos)
{
    __shared__ int2 buf[64][65];
    const uint32_t lane = threadIdx.x;
    const uint32_t g = blockIdx.x * 64 + lane;
    const bool active = g < n;
    RsTrack T;
    if (active)
        T = tr[ids[g]];
    double input_index = 0.0, ratio_inv = 0.0;
    uint64_t c = 0, total = active ? T.out_frames : 0;
    if (active)
        ratio_inv = __longlong_as_double((long long)T.D); // 1.0 / ratio (host double bits)
    // every lane runs the block's longest track's steps; shorter ones idle
    uint64_t steps = total;
    for (int o = 32; o > 0; o >>= 1)
        steps = max(steps, (uint64_t)__shfl_xor((unsigned long long)steps, o));
    for (uint64_t n0 = 0; n0 < steps; n0 += 64) {
        for (uint32_t k = 0; k < 64; ++k) {
            const uint64_t nn = n0 + k;
            int2 v = make_int2(0, 0);
            if (active && nn < total) {
                v.x = (int32_t)(uint32_t)c;
                v.y = (int32_t)__double2int_rn((input_index * T.float_increment) *
                                              (double)(1 << kShift));
                input_index = input_index + ratio_inv;
                // fmod_one (common.h:161-170) and the integer advance
                double r = input_index - rint(input_index);
                r = r < 0.0 ? r + 1.0 : r;
                c += (uint64_t)(int64_t)rint(input_index - r);
                input_index = r;
            }
            buf[lane][k] = v;
        }
        __syncthreads();
        // flush: track j's 64 entries, one lane each -> coalesced
        for (uint32_t j = 0; j < 64; ++j) {
            const uint32_t gj = blockIdx.x * 64 + j;
            if (gj >= n)
                break;
            const RsTrack Tj = tr[ids[gj]];
            const uint64_t nn = n0 + lane;
            if (nn < Tj.out_frames)
                pos[Tj.pos_base + nn] = buf[j][lane];
        }
        __syncthreads();
    }
}

// one half filter of calc_output_* (src_sinc.c:423-475): taps from the
// farthest in, while fi >= 0 (left) or fi > 0 (right), data index di
// stepping by +1 (left) or -1 (right) frames; the tap count is known up
// front, so the loop is counted and unrolled for ILP.  HOIST: the increment
// is a multiple of 4096 (ratio >= 1), so every tap of the half shares one
// interpolation fraction.  The coefficient c0 + fraction * (c1 - c0) is a
// fused multiply-add: fraction (12 bits) times the float difference (24
// bits) is exact in fp64, so the FMA rounds once exactly where the
// reference's separate multiply and add do.
// k_rs_phase's window layout for more than two channels: frame f's CH
// floats at f CH + f / 8 (one pad word after every 8 frames).  A wave's
// lanes read frames `lspan x ratio` apart (8 frames = 48 floats for 192 ->
// 48 kHz 5.1), which unpadded land on a few LDS banks (16-way conflicts,
// the kernel's largest stall); padded, the lane bases are 49 words apart,
// coprime with the bank count, and a frame's channels stay contiguous (one
// base per tap, the channels at immediate offsets).
template <int CH, bool PAD>
__device__ __forceinline__ uint32_t xframe(uint32_t f)
{
    return f * CH + (PAD ? f >> 3 : 0u);
}
// floats a window of `frames` frames occupies
__host__ __device__ inline size_t xpad_floats(size_t frames, int channels)
{
    return frames * channels + (channels > 2 ? frames / 8 + 1 : 0);
}

template <int CH, bool LEFT, bool HOIST, typename XT, bool PAD = false>
__device__ __forceinline__ void half_filter(const float *__restrict__ C, const XT *__restrict__ X,
                                            int32_t fi, int32_t inc, int32_t di,
                                            double (&acc)[CH])
{
    constexpr int32_t kMask = (1 << kShift) - 1;
    const double hfrac = (double)(fi & kMask) * (1.0 / 4096.0);
    const int32_t taps = LEFT ? fi / inc + 1 : (fi - 1) / inc + 1;
#pragma unroll 4
    for (int32_t j = 0; j < taps; ++j) {
        const double fraction = HOIST ? hfrac : (double)(fi & kMask) * (1.0 / 4096.0);
        const int32_t ix = fi >> kShift;
        const float c0 = C[ix], c1 = C[ix + 1];
        const double icoeff = __builtin_fma(fraction, (double)(c1 - c0), (double)c0);
#pragma unroll
        for (int k = 0; k < CH; ++k)
            acc[k] = acc[k] + icoeff * (double)X[xframe<CH, PAD>((uint32_t)di) + k];
        fi -= inc;
        di += LEFT ? 1 : -1;
    }
}

template <int CH, bool HOIST, typename XT>
__global__ __launch_bounds__(kChunk) void k_rs_filter(RsParams P, const RsTrack *__restrict__ tr,
                                                      const uint32_t *__restrict__ chunk_track,
                                                      const int2 *__restrict__ pos,
                                                      const uint32_t *__restrict__ table_bits,
                                                      const int32_t *__restrict__ in,
                                                      int32_t *__restrict__ out)
{
    extern __shared__ double lds_d[];
    float *C = reinterpret_cast<float *>(lds_d);                    // the coefficient table
    XT *X = reinterpret_cast<XT *>(lds_d + (((kTable + 3) & ~3) / 2)); // the chunk's input window
    for (uint32_t i = threadIdx.x; i < (uint32_t)kTable; i += blockDim.x)
        C[i] = __uint_as_float(table_bits[i]);
    __syncthreads();
    const int32_t max_fi = SRC_MEDIUM_HALF_LEN << kShift;
    for (uint32_t chunk = blockIdx.x; chunk < P.n_chunks; chunk += gridDim.x) {
        const uint32_t t = chunk_track[chunk];
        const RsTrack T = tr[t];
        const uint64_t n0 = (uint64_t)(chunk - T.chunk_base) * P.chunk;
        const uint64_t n_end = min(n0 + (uint64_t)P.chunk, T.out_frames);
        const int32_t inc = T.increment;
        // input window of the chunk: taps reach (max_fi / inc + 1) frames
        // either side of the centres
        const int64_t reach = (int64_t)(max_fi / inc) + 2;
        int64_t c_first, c_last;
        int32_t s_tmp;
        position(T, pos, n0, c_first, s_tmp);
        position(T, pos, n_end - 1, c_last, s_tmp);
        const int64_t w0 = c_first - reach, w1 = c_last + reach + 1; // [w0, w1)
        const uint32_t wn = (uint32_t)(w1 - w0);
        for (uint32_t i = threadIdx.x; i < wn * CH; i += blockDim.x) {
            const int64_t f = w0 + (int64_t)(i / CH);
            float v = 0.0f;
            if (f >= 0 && (uint64_t)f < T.in_frames)
                v = (float)in[T.in_base + (uint64_t)f * CH + (i % CH)] * P.inv_q;
            X[i] = (XT)v;
        }
        __syncthreads();
        const uint64_t n = n0 + threadIdx.x;
        if (n < n_end) {
            int64_t c;
            int32_t sfi;
            position(T, pos, n, c, sfi);
            double left[CH], right[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k)
                left[k] = right[k] = 0.0;
            int32_t cc = (max_fi - sfi) / inc;
            half_filter<CH, true, HOIST>(C, X, sfi + cc * inc, inc, (int32_t)(c - cc - w0), left);
            const int32_t fr = inc - sfi;
            cc = (max_fi - fr) / inc;
            half_filter<CH, false, HOIST>(C, X, fr + cc * inc, inc, (int32_t)(c + 1 + cc - w0),
                                          right);
            int32_t *o = out + T.out_base + n * CH;
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const float f = (float)(T.scale * (left[k] + right[k]));
                const float g = f * P.q;
                // (int) of a float: truncation; x86 gives INT_MIN out of range
                int32_t s = (g >= 2147483648.0f || g < -2147483648.0f || g != g)
                                ? (int32_t)0x80000000
                                : (int32_t)g;
                o[k] = s > P.hi ? P.hi : (s < P.lo ? P.lo : s);
            }
        }
        __syncthreads();
    }
}

// c0 + fraction * (c1 - c0) of filter index fi from the float table
__device__ __forceinline__ double interp_coeff(const float *__restrict__ C, int32_t fi)
{
    const double fraction = (double)(fi & ((1 << kShift) - 1)) * (1.0 / 4096.0);
    const int32_t ix = fi >> kShift;
    const float c0 = C[ix], c1 = C[ix + 1];
    return __builtin_fma(fraction, (double)(c1 - c0), (double)c0);
}

// output m's coefficient of one tap from the [tap][M] table: the M doubles
// of a tap are contiguous, so one ds_read_b128 (a wave-uniform address: an
// LDS broadcast) returns two outputs' coefficients
template <int M>
__device__ __forceinline__ void load_coefs(const double *__restrict__ p, double (&ic)[M])
{
    if constexpr (M % 2 == 0) {
#pragma unroll
        for (int m = 0; m < M; m += 2) {
            const double2 v = *(const double2 *)(p + m);
            ic[m] = v.x;
            ic[m + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int m = 0; m < M; ++m)
            ic[m] = p[m];
    }
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Tap windows of a phase group (M outputs of one lane row, the phases and
// centres lane 0 computed), relative to c_0: output m's left half is
// [dL_m, dc_m] ascending, its right half [dc_m + 1, top_m] descending, as
// calc_output_* walks them; the union windows are [sl0, sl1] and [sr0, sr1].
template <int M>
struct PhaseGeom {
    int32_t dL[M], fiL[M], nL[M], top[M], fiR[M], nR[M];
    int32_t sl0, sl1, sr0, sr1;
};

template <int M>
__device__ __forceinline__ void phase_geom(const int32_t (&sfi0)[M], const int32_t (&dc)[M],
                                           const bool (&valid)[M], int32_t inc, PhaseGeom<M> &q)
{
    const int32_t max_fi = SRC_MEDIUM_HALF_LEN << kShift;
    q.sl0 = 1 << 30;
    q.sl1 = -(1 << 30);
    q.sr0 = 1 << 30;
    q.sr1 = -(1 << 30);
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int32_t ccL = (max_fi - sfi0[m]) / inc;
        q.fiL[m] = sfi0[m] + ccL * inc;
        q.nL[m] = valid[m] ? q.fiL[m] / inc + 1 : 0;
        q.dL[m] = dc[m] - ccL;
        const int32_t frR = inc - sfi0[m];
        const int32_t ccR = (max_fi - frR) / inc;
        q.fiR[m] = frR + ccR * inc;
        q.nR[m] = valid[m] ? (q.fiR[m] - 1) / inc + 1 : 0;
        q.top[m] = dc[m] + 1 + ccR;
        if (valid[m]) {
            q.sl0 = min(q.sl0, q.dL[m]);
            q.sl1 = max(q.sl1, dc[m]);
            q.sr0 = min(q.sr0, dc[m] + 1);
            q.sr1 = max(q.sr1, q.top[m]);
        }
    }
}

// the group's zero-padded coefficient tables, [tap][M] (cL: left half over
// s = sl0 .. sl1, cR: right half over s = sr1 .. sr0), lanes over taps
template <int M>
__device__ __forceinline__ void phase_fill(const float *__restrict__ Cg, const PhaseGeom<M> &q,
                                           int32_t inc, uint32_t lane, double *__restrict__ cL,
                                           double *__restrict__ cR)
{
    const int32_t WL = q.sl1 - q.sl0 + 1, WR = q.sr1 - q.sr0 + 1;
    for (int32_t k = (int32_t)lane; k < WL; k += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t j = k + q.sl0 - q.dL[m];
            cL[k * M + m] = (j >= 0 && j < q.nL[m]) ? interp_coeff(Cg, q.fiL[m] - j * inc) : 0.0;
        }
    }
    for (int32_t k = (int32_t)lane; k < WR; k += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t j = q.top[m] - q.sr1 + k;
            cR[k * M + m] = (j >= 0 && j < q.nR[m]) ? interp_coeff(Cg, q.fiR[m] - j * inc) : 0.0;
        }
    }
}

// Phase tables of a ratio class, computed once per launch: group g of the
// first lane row (outputs M g .. M g + M - 1 of the class's first track)
// -> header (sl0, WL, sr1, WR, the M phases and relative centres it was
// built for) + left and right [tap][M] tables.  A filter item whose lane 0
// finds the same phases and centres (exact periodicity of the positions)
// copies them instead of evaluating c0 + fraction (c1 - c0) per tap.
constexpr uint32_t kTabHdr = 8; // header doubles (16 int32)

template <int M>
__global__ __launch_bounds__(64) void k_rs_phase_tab(const RsTrack *__restrict__ tr,
                                                     const uint32_t *__restrict__ class_track,
                                                     const int2 *__restrict__ pos,
                                                     const uint32_t *__restrict__ table_bits,
                                                     double *__restrict__ tabs, uint32_t G,
                                                     uint32_t wmax, uint64_t stride)
{
    const uint32_t g = blockIdx.x, cls = blockIdx.y, lane = threadIdx.x;
    const RsTrack T = tr[class_track[cls]];
    const uint32_t L = T.lspan;
    double *tb = tabs + ((uint64_t)cls * G + g) * stride;
    int32_t *th = reinterpret_cast<int32_t *>(tb);
    if (M * g >= L) {
        if (lane < 2 * kTabHdr)
            th[lane] = 0; // WL = 0: never taken
        return;
    }
    int64_t c[M];
    int32_t sfi[M], sfi0[M], dc[M];
    bool valid[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        valid[m] = M * g + m < L && (uint64_t)(M * g + m) < T.out_frames;
        position(T, pos, valid[m] ? M * g + m : M * g, c[m], sfi[m]);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        sfi0[m] = sfi[m];
        dc[m] = (int32_t)(c[m] - c[0]);
    }
    PhaseGeom<M> q;
    phase_geom<M>(sfi0, dc, valid, T.increment, q);
    bool all = true;
#pragma unroll
    for (int m = 0; m < M; ++m)
        all = all && valid[m];
    if (lane == 0) {
        th[0] = q.sl0;
        th[1] = all ? q.sl1 - q.sl0 + 1 : 0; // partial groups: never taken from the table
        th[2] = q.sr1;
        th[3] = all ? q.sr1 - q.sr0 + 1 : 0;
#pragma unroll
        for (int m = 0; m < M; ++m) {
            th[4 + m] = sfi0[m];
            th[4 + M + m] = dc[m];
        }
    }
    phase_fill<M>(reinterpret_cast<const float *>(table_bits), q, T.increment, lane, tb + kTabHdr,
                  tb + kTabHdr + (uint64_t)M * wmax);
}

// k_rs_phase's input window in LDS: floats, converted per tap (the same
// values widened to double once at staging measured 25.2 against 7.2 ms:
// twice the LDS per task halves the rows a task holds)
typedef float PhaseX;
constexpr size_t kPhaseXBytes = sizeof(PhaseX);

// The phase-sharing filter.  The output positions of a rational ratio
// repeat their fractional part every `period` = out_rate / gcd outputs, so
// outputs n, n + period, n + 2 period, ... have the same start filter index
// and the same interpolated coefficients.  A lane computes M consecutive
// outputs n0 .. n0 + M - 1 (their input windows overlap almost entirely);
// the 64 lanes of a wave are `lspan` outputs apart (a multiple of the
// period), so output m of every lane has the same phase.  Per work item
// (one group of M phases of one row of 64 lanes) the wave tabulates each
// output's coefficients once in LDS, zero-padded onto a common sample
// index: output m's left half is the taps x[c_m - ccL_m .. c_m] in order,
// so with s running over the union of the M windows, tap s of output m is
// coefficient (s - (c_m - ccL_m)) or 0.  Adding a zero product leaves an
// accumulator unchanged bit for bit (it starts at +0.0 and +0 + -0 = +0),
// and the nonzero taps keep the reference's order, so every output is
// exactly calc_output's.  One LDS read of a sample (and its float -> double
// conversion) then feeds M outputs' multiply + add per channel, and the
// coefficient reads are wave-uniform (LDS broadcast).  The right half runs
// the same way over s descending.  A task is 64 x lspan x rows consecutive
// outputs of one track, whose input window is staged in LDS as float
// x / 2^(bps-1).  Each lane still computes its own exact position; a work
// item whose lanes disagree on a phase (the fp64 recurrence drifting
// across a rounding boundary) takes the per-lane path with the
// coefficients read from the global table.
template <int CH, int M>
__global__ __launch_bounds__(1024) void k_rs_phase(RsParams P, const RsTrack *__restrict__ tr,
                                                  const uint2 *__restrict__ tasks,
                                                  uint32_t n_tasks, const int2 *__restrict__ pos,
                                                  const uint32_t *__restrict__ table_bits,
                                                  const int32_t *__restrict__ in,
                                                  int32_t *__restrict__ out, uint32_t wmax,
                                                  const double *__restrict__ tabs, uint32_t tab_G,
                                                  uint64_t tab_stride)
{
    extern __shared__ double lds_d[];
    constexpr bool PAD = CH > 2; // the window's layout (xpad)
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
    double *cL = lds_d + (size_t)wave * 2 * M * wmax; // [wmax][M] left, then right
    double *cR = cL + (size_t)M * wmax;
    PhaseX *X = reinterpret_cast<PhaseX *>(lds_d + (size_t)nwaves * 2 * M * wmax);
    const float *Cg = reinterpret_cast<const float *>(table_bits);
    const int32_t max_fi = SRC_MEDIUM_HALF_LEN << kShift;
    for (uint32_t task = blockIdx.x; task < n_tasks; task += gridDim.x) {
        const uint2 tk = tasks[task];
        const RsTrack T = tr[tk.x];
        const uint64_t B0 = (uint64_t)tk.y * T.span;
        const uint64_t Bend = min(B0 + T.span, T.out_frames);
        const int32_t inc = T.increment;
        const int64_t reach = (int64_t)(max_fi / inc) + 2;
        int64_t c_first, c_last;
        int32_t s_tmp;
        position(T, pos, B0, c_first, s_tmp);
        position(T, pos, Bend - 1, c_last, s_tmp);
        const int64_t w0 = c_first - reach;
        // wext more frames: a lane whose later outputs fall past the task's
        // end still reads their taps' samples (times zero coefficients for
        // its live outputs), so they must be finite -- staged, not stale LDS
        const uint32_t wn = (uint32_t)(c_last + reach + 1 - w0) + T.wext;
        // kStage loads in flight per thread before their conversions
        constexpr uint32_t kStage = 8;
        const uint32_t nx = wn * CH;
        for (uint32_t i0 = threadIdx.x; i0 < nx; i0 += kStage * blockDim.x) {
            int32_t v[kStage];
#pragma unroll
            for (uint32_t b = 0; b < kStage; ++b) {
                const uint32_t i = i0 + b * blockDim.x;
                const int64_t f = w0 + (int64_t)(i / CH);
                v[b] = 0;
                if (i < nx && f >= 0 && (uint64_t)f < T.in_frames)
                    v[b] = in[T.in_base + (uint64_t)f * CH + (i % CH)];
            }
#pragma unroll
            for (uint32_t b = 0; b < kStage; ++b) {
                const uint32_t i = i0 + b * blockDim.x;
                if (i < nx)
                    X[i + (PAD ? (i / CH) >> 3 : 0u)] = (PhaseX)((float)v[b] * P.inv_q);
            }
        }
        __syncthreads();
        const uint32_t L = T.lspan;
        const uint32_t G = (L + M - 1) / M; // phase groups per row
        const uint64_t row_len = 64ull * L;
        const uint32_t rows = (uint32_t)((Bend - B0 + row_len - 1) / row_len);
        for (uint32_t item = wave; item < rows * G; item += nwaves) {
            const uint32_t g = item % G;
            const uint64_t rbase = B0 + (uint64_t)(item / G) * row_len + (uint64_t)M * g;
            if (rbase >= Bend)
                continue; // wave-uniform: the last row's tail
            // output m of this lane; m is wave-valid when lane 0's is inside
            // the task and the group
            int64_t c[M];
            int32_t sfi[M];
            bool valid[M], active[M];
            bool uni = true;
#pragma unroll
            for (int m = 0; m < M; ++m) {
                valid[m] = (uint32_t)(M * g + m) < L && rbase + m < Bend;
                const uint64_t n = rbase + m + (uint64_t)L * lane;
                active[m] = valid[m] && n < Bend;
                position(T, pos, active[m] ? n : rbase + (valid[m] ? m : 0), c[m], sfi[m]);
            }
            // phases and relative centres uniform over the wave?
            int32_t sfi0[M];
            int32_t dc[M]; // c_m - c_0 (lane 0's)
#pragma unroll
            for (int m = 0; m < M; ++m) {
                sfi0[m] = __builtin_amdgcn_readfirstlane(sfi[m]);
                const int32_t d = (int32_t)(c[m] - c[0]);
                dc[m] = __builtin_amdgcn_readfirstlane(d);
                uni = uni && (!active[m] || (sfi[m] == sfi0[m] && d == dc[m]));
            }
            double left[M][CH], right[M][CH];
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int k = 0; k < CH; ++k)
                    left[m][k] = right[m][k] = 0.0;
            if (__all(uni)) {
                // the class's table for this group when lane 0's phases and
                // centres are the ones it was built for, else evaluated here
                const double *__restrict__ tb = tabs + ((uint64_t)T.cls * tab_G + g) * tab_stride;
                const int32_t *__restrict__ th = reinterpret_cast<const int32_t *>(tb);
                bool hit = th[1] != 0;
#pragma unroll
                for (int m = 0; m < M; ++m)
                    hit = hit && valid[m] && th[4 + m] == sfi0[m] && th[4 + M + m] == dc[m];
                int32_t sl0, sr1, WL, WR;
                if (hit) {
                    sl0 = th[0];
                    WL = th[1];
                    sr1 = th[2];
                    WR = th[3];
                    const double2 *__restrict__ gl = reinterpret_cast<const double2 *>(tb + kTabHdr);
                    const double2 *__restrict__ gr =
                        reinterpret_cast<const double2 *>(tb + kTabHdr + (uint64_t)M * wmax);
                    double2 *dl = reinterpret_cast<double2 *>(cL), *dr = reinterpret_cast<double2 *>(cR);
                    const int32_t nl = (WL * M + 1) / 2, nr = (WR * M + 1) / 2;
                    for (int32_t k = (int32_t)lane; k < max(nl, nr); k += 64) {
                        double2 a, b;
                        if (k < nl)
                            a = gl[k];
                        if (k < nr)
                            b = gr[k];
                        if (k < nl)
                            dl[k] = a;
                        if (k < nr)
                            dr[k] = b;
                    }
                } else {
                    PhaseGeom<M> q;
                    phase_geom<M>(sfi0, dc, valid, inc, q);
                    phase_fill<M>(Cg, q, inc, lane, cL, cR);
                    sl0 = q.sl0;
                    sr1 = q.sr1;
                    WL = q.sl1 - q.sl0 + 1;
                    WR = q.sr1 - q.sr0 + 1;
                }
                // wave-uniform by construction (the table header, or the
                // geometry of lane 0's phases): scalar loop control
                WL = __builtin_amdgcn_readfirstlane(WL);
                WR = __builtin_amdgcn_readfirstlane(WR);
                wave_lds_sync();
                const uint32_t fl = (uint32_t)(c[0] + sl0 - w0);
#pragma unroll 2
                for (int32_t k = 0; k < WL; ++k) {
                    double x[CH];
                    const PhaseX *xk = X + xframe<CH, PAD>(fl + (uint32_t)k);
#pragma unroll
                    for (int q = 0; q < CH; ++q)
                        x[q] = (double)xk[q];
                    double ic[M];
                    load_coefs<M>(cL + k * M, ic);
#pragma unroll
                    for (int m = 0; m < M; ++m) {
#pragma unroll
                        for (int q = 0; q < CH; ++q)
                            left[m][q] = left[m][q] + ic[m] * x[q];
                    }
                }
                const uint32_t fr0 = (uint32_t)(c[0] + sr1 - w0);
#pragma unroll 2
                for (int32_t k = 0; k < WR; ++k) {
                    double x[CH];
                    const PhaseX *xk = X + xframe<CH, PAD>(fr0 - (uint32_t)k);
#pragma unroll
                    for (int q = 0; q < CH; ++q)
                        x[q] = (double)xk[q];
                    double ic[M];
                    load_coefs<M>(cR + k * M, ic);
#pragma unroll
                    for (int m = 0; m < M; ++m) {
#pragma unroll
                        for (int q = 0; q < CH; ++q)
                            right[m][q] = right[m][q] + ic[m] * x[q];
                    }
                }
                wave_lds_sync(); // the tables are rewritten by the next item
            } else {
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    if (!valid[m])
                        continue;
                    const int32_t ccl = (max_fi - sfi[m]) / inc;
                    half_filter<CH, true, false, PhaseX, PAD>(Cg, X, sfi[m] + ccl * inc, inc,
                                                 (int32_t)(c[m] - ccl - w0), left[m]);
                    const int32_t fr = inc - sfi[m];
                    const int32_t ccr = (max_fi - fr) / inc;
                    half_filter<CH, false, false, PhaseX, PAD>(Cg, X, fr + ccr * inc, inc,
                                                  (int32_t)(c[m] + 1 + ccr - w0), right[m]);
                }
            }
#pragma unroll
            for (int m = 0; m < M; ++m) {
                if (!active[m])
                    continue;
                int32_t *o = out + T.out_base + (rbase + m + (uint64_t)L * lane) * CH;
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const float f = (float)(T.scale * (left[m][k] + right[m][k]));
                    const float gq = f * P.q;
                    int32_t sv = (gq >= 2147483648.0f || gq < -2147483648.0f || gq != gq)
                                     ? (int32_t)0x80000000
                                     : (int32_t)gq;
                    o[k] = sv > P.hi ? P.hi : (sv < P.lo ? P.lo : sv);
                }
            }
        }
        __syncthreads();
    }
}

// outputs per lane of k_rs_phase: as many as the accumulators allow
template <int CH>
constexpr int phase_m() { return CH <= 2 ? 5 : 2; }

// ------------------------------------------------------------------ host
thread_local std::string g_rs_err;

atg_status rsfail(atg_status s, const std::string &m)
{
    g_rs_err = m;
    return s;
}

#define RSHIP(expr)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return rsfail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

double fmod_one(double x)
{
    double r = x - (double)std::lrint(x);
    return r < 0.0 ? r + 1.0 : r;
}

// the per-track converter constants (sinc_set_converter + *_vari_process)
struct Conv {
    double ratio, float_increment, scale, terminate, inv;
    int32_t increment;
    int mode;
    uint64_t D;
    uint32_t half_frames; // half_filter_chan_len / channels
};

Conv make_conv(uint32_t in_rate, uint32_t out_rate)
{
    Conv v;
    v.ratio = (double)out_rate / (double)in_rate;
    const int index_inc = SRC_MEDIUM_INCREMENT;
    v.float_increment = index_inc * 1.0;
    if (v.ratio < 1.0)
        v.float_increment = index_inc * v.ratio;
    v.increment = (int32_t)std::lrint(v.float_increment * 4096.0);
    v.scale = v.float_increment / index_inc;
    v.terminate = 1.0 / v.ratio + 1e-20;
    v.inv = 1.0 / v.ratio;
    double count = (SRC_MEDIUM_HALF_LEN + 2.0) / index_inc;
    if (v.ratio < 1.0)
        count /= v.ratio;
    v.half_frames = (uint32_t)(std::lrint(count) + 1);
    // exact closed forms of the position recurrence (file comment)
    const double d = v.inv;
    v.mode = POS_TABLE;
    v.D = 0;
    if (d >= 0.5 && d < 1.0) {
        const double scaled = std::ldexp(d, 53);
        const uint64_t Di = (uint64_t)scaled;
        if ((double)Di == scaled && (Di & 1u) == 0) {
            v.mode = POS_CLOSED_FRAC;
            v.D = Di;
        }
    } else if (d >= 1.0 && d == std::floor(d) && d < 4294967296.0) {
        v.mode = POS_CLOSED_INT;
        v.D = (uint64_t)d;
    }
    if (v.mode == POS_TABLE) {
        uint64_t bits;
        std::memcpy(&bits, &d, 8);
        v.D = bits; // the serial kernel reads 1/ratio from here
    }
    return v;
}

// host replica of the position of output n for the closed forms
void host_position(const Conv &v, uint64_t n, uint64_t &c, double &frac)
{
    if (v.mode == POS_CLOSED_FRAC) {
        const unsigned __int128 p = (unsigned __int128)n * v.D;
        c = (uint64_t)(p >> 53);
        frac = std::ldexp((double)(uint64_t)(p & ((1ull << 53) - 1ull)), -53);
    } else {
        c = n * v.D;
        frac = 0.0;
    }
}

// The reference's control flow with the data left out: Resampler.read()
// (pcmconverter.c:439-495) around src_process (samplerate.c:122-183),
// sinc_*_vari_process (src_sinc.c:478-568) and prepare_data (:1135-1205),
// tracking only buffer positions.  It gives the frame count of every read()
// and the exact end of the stream: the termination test of :532-535 adds
// the fractional position to the circular-buffer index b_current, so its
// rounding depends on the buffer history, not just on the output index.
struct SrcSim {
    int64_t ch, b_len, half;
    double inv, terminate;
    int64_t b_current = 0, b_end = 0, b_real_end = -1;
    double input_index = 0.0; // last_position

    SrcSim(const Conv &v, uint32_t channels)
    {
        ch = channels;
        const int64_t frames = std::max<int64_t>(
            std::lrint(2.5 * SRC_MEDIUM_HALF_LEN / (SRC_MEDIUM_INCREMENT * 1.0) * 256.0), 4096);
        b_len = frames * ch;
        half = ch * (int64_t)v.half_frames;
        inv = v.inv;
        terminate = v.terminate;
    }

    // prepare_data; in_count/in_used in samples
    void prepare(int64_t in_count, int64_t &in_used, bool eoi)
    {
        if (b_real_end >= 0)
            return;
        int64_t len;
        if (b_current == 0) {
            len = b_len - 2 * half;
            b_current = b_end = half;
        } else if (b_end + half + ch < b_len) {
            len = std::max<int64_t>(b_len - b_current - half, 0);
        } else {
            len = b_end - b_current;
            b_current = half;
            b_end = b_current + len;
            len = std::max<int64_t>(b_len - b_current - half, 0);
        }
        len = std::min(in_count - in_used, len);
        len -= len % ch;
        b_end += len;
        in_used += len;
        if (in_used == in_count && b_end - b_current < 2 * half && eoi) {
            if (b_len - b_end < half + 5) {
                len = b_end - b_current;
                b_current = half;
                b_end = b_current + len;
            }
            b_real_end = b_end;
            len = half + 5;
            if (b_end + len > b_len)
                len = b_len - b_end;
            b_end += len;
        }
    }

    // one src_process call over in_frames pending frames with room for
    // out_frames outputs -> (frames used, frames generated)
    void process(uint64_t in_frames, uint64_t out_frames, bool eoi, uint64_t &used,
                 uint64_t &gen)
    {
        const int64_t in_count = (int64_t)in_frames * ch, out_count = (int64_t)out_frames * ch;
        int64_t in_used = 0, out_gen = 0;
        while (out_gen < out_count) {
            int64_t sih = (b_end - b_current + b_len) % b_len;
            if (sih <= half) {
                prepare(in_count, in_used, eoi);
                sih = (b_end - b_current + b_len) % b_len;
                if (sih <= half)
                    break;
            }
            if (b_real_end >= 0 &&
                (double)b_current + input_index + terminate >= (double)b_real_end)
                break;
            out_gen += ch;
            input_index += inv;
            const double rem = fmod_one(input_index);
            b_current = (b_current + ch * (int64_t)std::lrint(input_index - rem)) % b_len;
            input_index = rem;
        }
        used = (uint64_t)(in_used / ch);
        gen = (uint64_t)(out_gen / ch);
    }
};

// Resampler.read() frame counts for a source whose read(4096) calls return
// reads[0..n_reads) (NULL: 4096-frame reads of `frames`); every count is
// passed to `sink` (the final 0 included).  Returns the total.
template <class Sink>
uint64_t simulate_reads(const Conv &v, uint32_t ch, uint64_t frames, const uint32_t *reads,
                        uint64_t n_reads, Sink sink)
{
    SrcSim sim(v, ch);
    uint64_t max_frames = (uint64_t)(uint32_t)std::ceil(4096 * v.ratio);
    uint64_t pending = 0, r = 0, fed = 0, total = 0;
    for (;;) {
        uint64_t out = 0;
        bool eoi;
        do {
            uint64_t got;
            if (reads)
                got = r < n_reads ? reads[r++] : 0;
            else
                got = std::min<uint64_t>(4096, frames - fed);
            fed += got;
            pending += got;
            eoi = pending == 0;
            uint64_t used, gen;
            sim.process(pending, max_frames, eoi, used, gen);
            pending -= used;
            if (pending > 0)
                max_frames += max_frames;
            out += gen;
        } while (out == 0 && !eoi);
        sink(out);
        total += out;
        if (out == 0)
            return total;
    }
}

// the closed-form position of output n (POS_CLOSED_*), exactly
void host_position(const Conv &v, uint64_t n, uint64_t &c, uint64_t &S)
{
    if (v.mode == POS_CLOSED_FRAC) {
        const unsigned __int128 p = (unsigned __int128)n * v.D;
        c = (uint64_t)(p >> 53);
        S = (uint64_t)(p & ((1ull << 53) - 1ull));
    } else {
        c = n * v.D;
        S = 0;
    }
}

// output frame count.  Closed forms: the first n with
// ch*c_n + frac_n + 1/ratio >= ch*frames (the sequence increases), found by
// bisection in exact integer arithmetic; when that comparison is within
// rounding distance of a tie (the reference evaluates it in doubles on a
// buffer-relative index), and for ratios without a closed form, the count
// comes from the control-flow simulation.
uint64_t output_frames(const Conv &v, uint32_t ch, uint64_t frames, const uint32_t *reads,
                       uint64_t n_reads)
{
    if (v.mode == POS_TABLE)
        return simulate_reads(v, ch, frames, reads, n_reads, [](uint64_t) {});
    // margin(n) = ch*(frames - c_n) - (frac_n + d) in units of 2^-53 (FRAC)
    // or of 1 (INT): terminated iff margin <= 0
    auto margin = [&](uint64_t n) -> __int128 {
        uint64_t c, S;
        host_position(v, n, c, S);
        const __int128 k = (__int128)ch * ((__int128)frames - (__int128)c);
        if (v.mode == POS_CLOSED_FRAC)
            return (k << 53) - (__int128)S - (__int128)v.D;
        return k - (__int128)v.D;
    };
    uint64_t lo = 0, hi = (uint64_t)((double)frames * v.ratio) + 64;
    while (margin(hi) > 0)
        hi *= 2;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (margin(mid) <= 0)
            hi = mid;
        else
            lo = mid + 1;
    }
    if (v.mode == POS_CLOSED_FRAC) {
        // the reference's sum b_current + frac + 1/ratio (b_current < b_len
        // < 2^20) rounds by at most 2^-33: a margin within 2^-29 of zero
        // is settled by the simulation
        const __int128 tol = (__int128)1 << 24;
        const __int128 m0 = margin(lo), m1 = lo ? margin(lo - 1) : tol + 1;
        if ((m0 > -tol && m0 <= tol) || (m1 > -tol && m1 <= tol))
            return simulate_reads(v, ch, frames, reads, n_reads, [](uint64_t) {});
    }
    return lo;
}

struct FilterArgs {
    RsParams P;
    const RsTrack *tr;
    const uint32_t *chunk_track;
    const int2 *pos;
    const uint32_t *table;
    const int32_t *in;
    int32_t *out;
};

template <int CH>
void launch_filter(const FilterArgs &A, bool hoist, bool xd, unsigned grid, unsigned block,
                   size_t lds, hipStream_t s)
{
#define RS_GO(H, XT)                                                                           \
    hipLaunchKernelGGL((k_rs_filter<CH, H, XT>), dim3(grid), dim3(block), lds, s, A.P, A.tr,   \
                       A.chunk_track, A.pos, A.table, A.in, A.out)
    if (hoist && xd)
        RS_GO(true, double);
    else if (hoist)
        RS_GO(true, float);
    else if (xd)
        RS_GO(false, double);
    else
        RS_GO(false, float);
#undef RS_GO
}

// threads per k_rs_phase block: its waves share the block's input window.
// <= 2 channels: 16 waves (4 per SIMD) over M = 5, 32 groups of a 160-output
// lane span = 2 items per wave (config 3: 7.86 -> 7.34 ms against 8 waves,
// M = 4); more channels: 8 waves (the 6-channel config-5 resample ran 16.1
// -> 18.2 ms at 16)
constexpr unsigned phase_threads(uint32_t channels) { return channels <= 2 ? 1024u : 512u; }

struct PhaseTabs {
    const uint32_t *class_track; // a track of each ratio class
    uint32_t n_classes, G;       // classes, phase groups per class
    double *tabs;
    uint64_t stride;             // doubles per group table
};

template <int CH>
void launch_phase(const FilterArgs &A, const uint2 *tasks, uint32_t n_tasks, uint32_t wmax,
                  unsigned grid, size_t lds, const PhaseTabs &pt, hipStream_t s)
{
    constexpr int M = phase_m<CH>();
    hipLaunchKernelGGL((k_rs_phase_tab<M>), dim3(pt.G, pt.n_classes), dim3(64), 0, s, A.tr,
                       pt.class_track, A.pos, A.table, pt.tabs, pt.G, wmax, pt.stride);
    hipLaunchKernelGGL((k_rs_phase<CH, M>), dim3(grid), dim3(phase_threads(CH)), lds, s, A.P, A.tr,
                       tasks, n_tasks, A.pos, A.table, A.in, A.out, wmax,
                       (const double *)pt.tabs, pt.G, pt.stride);
}

template <int CH>
hipError_t set_lds_attr()
{
    const hipFuncAttribute a = hipFuncAttributeMaxDynamicSharedMemorySize;
    hipError_t e = hipFuncSetAttribute((const void *)k_rs_phase<CH, phase_m<CH>()>, a, 160 * 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)k_rs_filter<CH, true, double>, a, 160 * 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)k_rs_filter<CH, true, float>, a, 160 * 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)k_rs_filter<CH, false, double>, a, 160 * 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)k_rs_filter<CH, false, float>, a, 160 * 1024);
    return e;
}

struct RsCtx {
    void *tracks = nullptr, *chunk_track = nullptr, *pos = nullptr, *table = nullptr,
         *ids = nullptr, *ptasks = nullptr, *ctrack = nullptr, *tabs = nullptr;
    size_t cap_tracks = 0, cap_chunks = 0, cap_pos = 0, cap_ids = 0, cap_ptasks = 0,
           cap_ctrack = 0, cap_tabs = 0;
    bool table_up = false;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    float ms[2] = {0.0f, 0.0f};
};
constexpr int kMaxDev = 64;
RsCtx g_rs[kMaxDev];

hipError_t grow(void *&p, size_t &cap, size_t bytes)
{
    if (p && bytes <= cap)
        return hipSuccess;
    if (p)
        (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess)
        cap = want;
    return e;
}

} // namespace

extern "C" {

const char *atg_resample_last_error(void) { return g_rs_err.c_str(); }

uint64_t atg_resample_output_frames(uint64_t in_frames, uint32_t channels, uint32_t in_rate,
                                    uint32_t out_rate)
{
    if (!in_rate || !out_rate || !channels)
        return 0;
    return output_frames(make_conv(in_rate, out_rate), channels, in_frames, nullptr, 0);
}

atg_status atg_resample_device(const atg_rs_track *tracks, uint32_t n, uint32_t channels,
                               uint32_t bits_per_sample, const int32_t *d_in, int32_t *d_out,
                               uint64_t out_cap_samples, uint64_t *out_offsets,
                               uint64_t *out_frames, void *stream)
{
    if ((!tracks && n) || !out_offsets || !out_frames)
        return rsfail(ATG_ERR_INVALID, "NULL argument");
    if (channels < 1 || channels > 8)
        return rsfail(ATG_ERR_UNSUPPORTED, "channels must be 1..8");
    if (bits_per_sample < 1 || bits_per_sample > 24)
        return rsfail(ATG_ERR_UNSUPPORTED, "bits per sample must be 1..24");
    hipStream_t s = (hipStream_t)stream;
    int dev = 0;
    RSHIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev)
        return rsfail(ATG_ERR_UNSUPPORTED, "device index too large");
    RsCtx &X = g_rs[dev];
    std::vector<RsTrack> tr(n);
    std::vector<uint32_t> chunk_track, serial;
    // outputs per block iteration: the LDS holds the table plus the input
    // window of one chunk (chunk / ratio frames plus the taps either side)
    std::vector<Conv> conv(n);
    for (uint32_t t = 0; t < n; ++t) {
        const atg_rs_track &a = tracks[t];
        if (!a.in_rate || !a.out_rate)
            return rsfail(ATG_ERR_INVALID, "sample rates must be positive");
        conv[t] = make_conv(a.in_rate, a.out_rate);
        if (conv[t].ratio > 256.0 || conv[t].ratio < 1.0 / 256.0) // is_bad_src_ratio
            return rsfail(ATG_ERR_INVALID, "SRC ratio outside [1/256, 256]");
    }
    // Phase-sharing plan (k_rs_phase): a track whose rational ratio repeats
    // its phases every `period` outputs goes there when a task of 64 x lspan
    // outputs fits the LDS with its input window and the per-wave
    // coefficient tables; the rest go to the per-output kernel k_rs_filter.
    const int32_t max_fi = SRC_MEDIUM_HALF_LEN << kShift;
    const size_t kLds = 160 * 1024;
    const uint32_t pm = channels <= 2 ? 5u : 2u; // phase_m<CH>()
    const size_t waves = phase_threads(channels) / 64;
    std::vector<uint32_t> per(n, 0), rows(n, 0), lspan(n, 0);
    std::vector<char> phase(n, 0);
    uint32_t wmax = 0;
    for (int it = 0; it < 2; ++it) {
        uint32_t wm = 0;
        for (uint32_t t = 0; t < n; ++t) {
            const uint64_t g = std::gcd((uint64_t)tracks[t].in_rate, (uint64_t)tracks[t].out_rate);
            const uint64_t p_out = tracks[t].out_rate / g, q_in = tracks[t].in_rate / g;
            const uint64_t reach = (uint64_t)(max_fi / conv[t].increment) + 2;
            const uint64_t step = (tracks[t].in_rate + tracks[t].out_rate - 1) / tracks[t].out_rate;
            // even: the [tap][M] tables stay 16-byte aligned for odd M
            const uint32_t wm_t = (uint32_t)(reach + (pm - 1) * step + 2 + 1) & ~1u;
            const size_t coef = waves * 2 * pm * std::max<uint32_t>(wmax, wm_t) * sizeof(double);
            phase[t] = 0;
            if (p_out > 65536)
                continue;
            const uint64_t L = p_out * ((pm + p_out - 1) / p_out);
            uint64_t r = 0;
            for (uint64_t R = 1; R <= 64; R *= 2) {
                const size_t win =
                    xpad_floats((size_t)(64 * (L / p_out) * q_in * R + 2 * reach + 8 +
                                         (pm - 1) * step + 2), (int)channels) *
                    kPhaseXBytes;
                if (coef + win > kLds)
                    break;
                r = R;
                if (64 * L * R >= std::max<uint64_t>(tracks[t].pcm_frames, 1) * 2)
                    break; // one task already covers the track
            }
            if (!r)
                continue;
            phase[t] = 1;
            per[t] = (uint32_t)p_out;
            lspan[t] = (uint32_t)L;
            rows[t] = (uint32_t)r;
            wm = std::max<uint32_t>(wm, wm_t);
        }
        if (wm <= wmax)
            break;
        wmax = wm;
    }
    // k_rs_filter: the window as doubles when a chunk of >= 512 outputs fits
    // (no conversion per tap), else as floats with the largest chunk that fits
    double min_ratio = 1e300;
    int32_t min_inc = 1 << 30;
    bool hoist = true;
    for (uint32_t t = 0; t < n; ++t) {
        if (phase[t])
            continue;
        min_ratio = std::min(min_ratio, conv[t].ratio);
        min_inc = std::min(min_inc, conv[t].increment);
        hoist = hoist && (conv[t].increment & ((1 << kShift) - 1)) == 0;
    }
    uint32_t chunk = 0;
    size_t lds = 0;
    bool xd = false;
    if (min_inc == (1 << 30)) { // every track goes to k_rs_phase
        chunk = kChunk;
        min_inc = 1 << 20;
        min_ratio = 1.0;
    }
    for (int pass = 0; pass < 2 && !chunk; ++pass) {
        const size_t xsz = pass == 0 ? sizeof(double) : sizeof(float);
        for (uint32_t ck = kChunk; ck >= (pass == 0 ? 512u : 64u); ck /= 2) {
            const uint64_t reach = (uint64_t)((SRC_MEDIUM_HALF_LEN << kShift) / min_inc) + 2;
            const uint64_t wn = (uint64_t)std::ceil(ck / min_ratio) + 2 * reach + 4;
            const size_t need = sizeof(float) * ((kTable + 3) & ~3) + xsz * wn * channels;
            if (need <= kLds) {
                chunk = ck;
                lds = need;
                xd = pass == 0;
                break;
            }
        }
    }
    if (!chunk)
        return rsfail(ATG_ERR_UNSUPPORTED, "resampling ratio too low for the LDS window");
    std::vector<uint2> ptasks;
    size_t lds_phase = 0;
    // ratio classes of the phase tracks (one table set each)
    std::vector<uint32_t> class_track;
    std::vector<std::pair<uint64_t, uint32_t>> class_key; // (in_rate << 32 | out_rate, class)
    uint32_t tab_G = 0;
    uint64_t out = 0, posn = 0;
    for (uint32_t t = 0; t < n; ++t) {
        const atg_rs_track &a = tracks[t];
        const Conv &v = conv[t];
        RsTrack &T = tr[t];
        T.in_base = a.pcm_offset * channels;
        T.in_frames = a.pcm_frames;
        T.out_frames = output_frames(v, channels, a.pcm_frames, a.reads, a.n_reads);
        T.out_base = out * channels;
        T.float_increment = v.float_increment;
        T.scale = v.scale;
        T.increment = v.increment;
        T.mode = v.mode;
        T.D = v.D;
        T.pos_base = 0;
        T.span = 0;
        T.period = per[t];
        T.lspan = lspan[t];
        T.wext = (pm - 1) * (uint32_t)((a.in_rate + a.out_rate - 1) / a.out_rate) + 2;
        T.cls = 0;
        if (v.mode == POS_TABLE) {
            T.pos_base = posn;
            posn += T.out_frames;
            serial.push_back(t);
        }
        T.chunk_base = chunk_track.size();
        if (phase[t]) {
            const uint64_t key = ((uint64_t)a.in_rate << 32) | a.out_rate;
            uint32_t cls = (uint32_t)class_track.size();
            for (const auto &kc : class_key)
                if (kc.first == key)
                    cls = kc.second;
            if (cls == class_track.size()) {
                class_key.emplace_back(key, cls);
                class_track.push_back(t);
                tab_G = std::max<uint32_t>(tab_G, (lspan[t] + pm - 1) / pm);
            }
            T.cls = cls;
            T.span = 64ull * lspan[t] * rows[t];
            for (uint64_t k = 0; k * T.span < T.out_frames; ++k)
                ptasks.push_back(make_uint2(t, (uint32_t)k));
            const uint64_t g = std::gcd((uint64_t)a.in_rate, (uint64_t)a.out_rate);
            const uint64_t reach = (uint64_t)(max_fi / v.increment) + 2;
            lds_phase = std::max(lds_phase, waves * 2 * pm * wmax * sizeof(double) +
                                                xpad_floats((size_t)(64 * (lspan[t] / per[t]) *
                                                                         (a.in_rate / g) * rows[t] +
                                                                     2 * reach + 8 + T.wext),
                                                            (int)channels) *
                                                    kPhaseXBytes);
        } else {
            for (uint64_t k = 0; k < (T.out_frames + chunk - 1) / chunk; ++k)
                chunk_track.push_back(t);
        }
        out_offsets[t] = out;
        out_frames[t] = T.out_frames;
        out += T.out_frames;
    }
    if (out * channels > out_cap_samples)
        return rsfail(ATG_ERR_CAPACITY, "output buffer too small (atg_resample_output_frames)");
    if (!X.table_up) {
        RSHIP(hipMalloc(&X.table, sizeof(SRC_MEDIUM_BITS)));
        RSHIP(hipMemcpy(X.table, SRC_MEDIUM_BITS, sizeof(SRC_MEDIUM_BITS), hipMemcpyHostToDevice));
        for (int k = 0; k < 3; ++k)
            RSHIP(hipEventCreate(&X.ev[k]));
        RSHIP(set_lds_attr<1>());
        RSHIP(set_lds_attr<2>());
        RSHIP(set_lds_attr<3>());
        RSHIP(set_lds_attr<4>());
        RSHIP(set_lds_attr<5>());
        RSHIP(set_lds_attr<6>());
        RSHIP(set_lds_attr<7>());
        RSHIP(set_lds_attr<8>());
        X.table_up = true;
    }
    RSHIP(grow(X.tracks, X.cap_tracks, sizeof(RsTrack) * std::max<uint32_t>(n, 1)));
    RSHIP(grow(X.chunk_track, X.cap_chunks, sizeof(uint32_t) * std::max<size_t>(chunk_track.size(), 1)));
    RSHIP(grow(X.pos, X.cap_pos, sizeof(int2) * std::max<uint64_t>(posn, 1)));
    RSHIP(grow(X.ids, X.cap_ids, sizeof(uint32_t) * std::max<size_t>(serial.size(), 1)));
    RSHIP(grow(X.ptasks, X.cap_ptasks, sizeof(uint2) * std::max<size_t>(ptasks.size(), 1)));
    const uint64_t tab_stride = kTabHdr + 2ull * pm * wmax;
    RSHIP(grow(X.ctrack, X.cap_ctrack, sizeof(uint32_t) * std::max<size_t>(class_track.size(), 1)));
    RSHIP(grow(X.tabs, X.cap_tabs,
               sizeof(double) * std::max<uint64_t>(tab_stride * tab_G * class_track.size(), 1)));
    if (!class_track.empty())
        RSHIP(hipMemcpyAsync(X.ctrack, class_track.data(), sizeof(uint32_t) * class_track.size(),
                             hipMemcpyHostToDevice, s));
    if (!ptasks.empty())
        RSHIP(hipMemcpyAsync(X.ptasks, ptasks.data(), sizeof(uint2) * ptasks.size(),
                             hipMemcpyHostToDevice, s));
    if (n)
        RSHIP(hipMemcpyAsync(X.tracks, tr.data(), sizeof(RsTrack) * n, hipMemcpyHostToDevice, s));
    if (!chunk_track.empty())
        RSHIP(hipMemcpyAsync(X.chunk_track, chunk_track.data(),
                             sizeof(uint32_t) * chunk_track.size(), hipMemcpyHostToDevice, s));
    RSHIP(hipEventRecord(X.ev[0], s));
    if (!serial.empty()) {
        RSHIP(hipMemcpyAsync(X.ids, serial.data(), sizeof(uint32_t) * serial.size(),
                             hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_rs_positions, dim3((unsigned)((serial.size() + 63) / 64)),
                           dim3(64), 0, s, (const RsTrack *)X.tracks,
                           (const uint32_t *)X.ids, (uint32_t)serial.size(), (int2 *)X.pos);
        RSHIP(hipGetLastError());
    }
    RsParams P;
    P.ch = channels;
    P.bps = bits_per_sample;
    P.n_tracks = n;
    P.n_chunks = (uint32_t)chunk_track.size();
    P.q = (float)(1u << (bits_per_sample - 1));
    P.inv_q = 1.0f / P.q;
    P.lo = -(int32_t)(1u << (bits_per_sample - 1));
    P.hi = (int32_t)(1u << (bits_per_sample - 1)) - 1;
    P.chunk = chunk;
    RSHIP(hipEventRecord(X.ev[1], s));
    if (P.n_chunks) {
        const unsigned grid = std::min<uint32_t>(P.n_chunks, 256u);
        const FilterArgs A{P, (const RsTrack *)X.tracks, (const uint32_t *)X.chunk_track,
                           (const int2 *)X.pos, (const uint32_t *)X.table, d_in, d_out};
        switch (channels) {
        case 1: launch_filter<1>(A, hoist, xd, grid, chunk, lds, s); break;
        case 2: launch_filter<2>(A, hoist, xd, grid, chunk, lds, s); break;
        case 3: launch_filter<3>(A, hoist, xd, grid, chunk, lds, s); break;
        case 4: launch_filter<4>(A, hoist, xd, grid, chunk, lds, s); break;
        case 5: launch_filter<5>(A, hoist, xd, grid, chunk, lds, s); break;
        case 6: launch_filter<6>(A, hoist, xd, grid, chunk, lds, s); break;
        case 7: launch_filter<7>(A, hoist, xd, grid, chunk, lds, s); break;
        default: launch_filter<8>(A, hoist, xd, grid, chunk, lds, s); break;
        }
        RSHIP(hipGetLastError());
    }
    if (!ptasks.empty()) {
        const FilterArgs A{P, (const RsTrack *)X.tracks, (const uint32_t *)X.chunk_track,
                           (const int2 *)X.pos, (const uint32_t *)X.table, d_in, d_out};
        const unsigned per_cu = lds_phase <= kLds / 2 ? 2u : 1u;
        const unsigned grid = (unsigned)std::min<size_t>(ptasks.size(), 256u * per_cu);
        const uint2 *tk = (const uint2 *)X.ptasks;
        const uint32_t nt = (uint32_t)ptasks.size();
        const PhaseTabs pt{(const uint32_t *)X.ctrack, (uint32_t)class_track.size(), tab_G,
                           (double *)X.tabs, tab_stride};
        switch (channels) {
        case 1: launch_phase<1>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 2: launch_phase<2>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 3: launch_phase<3>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 4: launch_phase<4>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 5: launch_phase<5>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 6: launch_phase<6>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        case 7: launch_phase<7>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        default: launch_phase<8>(A, tk, nt, wmax, grid, lds_phase, pt, s); break;
        }
        RSHIP(hipGetLastError());
    }
    RSHIP(hipEventRecord(X.ev[2], s));
    RSHIP(hipStreamSynchronize(s));
    X.ms[0] = X.ms[1] = 0.0f;
    (void)hipEventElapsedTime(&X.ms[0], X.ev[0], X.ev[1]);
    (void)hipEventElapsedTime(&X.ms[1], X.ev[1], X.ev[2]);
    return ATG_OK;
}

int atg_resample_kernel_times(const char **names, float *ms, int cap)
{
    static const char *kNames[2] = {"rs_positions", "rs_filter"};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev)
        return 0;
    for (int k = 0; k < 2 && k < cap; ++k) {
        if (names)
            names[k] = kNames[k];
        if (ms)
            ms[k] = g_rs[dev].ms[k];
    }
    return 2;
}

atg_status atg_resample_host(int device, const atg_rs_track *tracks, uint32_t n,
                             uint32_t channels, uint32_t bits_per_sample, const int32_t *in,
                             uint64_t in_samples, int32_t *out, uint64_t out_cap_samples,
                             uint64_t *out_offsets, uint64_t *out_frames)
{
    RSHIP(hipSetDevice(device));
    if (channels < 1 || channels > 8)
        return rsfail(ATG_ERR_UNSUPPORTED, "channels must be 1..8");
    uint64_t total = 0;
    for (uint32_t t = 0; t < n; ++t) {
        if (!tracks[t].in_rate || !tracks[t].out_rate)
            return rsfail(ATG_ERR_INVALID, "sample rates must be positive");
        total += output_frames(make_conv(tracks[t].in_rate, tracks[t].out_rate), channels,
                               tracks[t].pcm_frames, tracks[t].reads, tracks[t].n_reads);
    }
    if (total * channels > out_cap_samples)
        return rsfail(ATG_ERR_CAPACITY, "output buffer too small (atg_resample_output_frames)");
    int32_t *d_in = nullptr, *d_out = nullptr;
    RSHIP(hipMalloc(&d_in, std::max<uint64_t>(in_samples, 1) * 4));
    hipError_t e = hipMalloc(&d_out, std::max<uint64_t>(total * channels, 1) * 4);
    if (e != hipSuccess) {
        (void)hipFree(d_in);
        return rsfail(ATG_ERR_NOMEM, hipGetErrorString(e));
    }
    atg_status st = ATG_OK;
    if (in_samples && hipMemcpy(d_in, in, in_samples * 4, hipMemcpyHostToDevice) != hipSuccess)
        st = rsfail(ATG_ERR_DEVICE, "hipMemcpy input");
    if (st == ATG_OK)
        st = atg_resample_device(tracks, n, channels, bits_per_sample, d_in, d_out,
                                 total * channels, out_offsets, out_frames, nullptr);
    if (st == ATG_OK && total &&
        hipMemcpy(out, d_out, total * channels * 4, hipMemcpyDeviceToHost) != hipSuccess)
        st = rsfail(ATG_ERR_DEVICE, "hipMemcpy output");
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return st;
}

// the frame counts Resampler.read() returns, one per call (pcmconverter.c
// :439-495 over src_process): `reads` are the frame counts the wrapped
// reader's read(4096) calls returned
int64_t atg_resample_read_sizes(uint64_t in_frames, uint32_t channels, uint32_t in_rate,
                                uint32_t out_rate, const uint32_t *reads, uint64_t n_reads,
                                uint32_t *sizes, uint64_t cap)
{
    if (!in_rate || !out_rate || !channels || channels > 8)
        return -1;
    const Conv v = make_conv(in_rate, out_rate);
    int64_t k = 0;
    simulate_reads(v, channels, in_frames, reads, n_reads, [&](uint64_t n) {
        if (sizes && (uint64_t)k < cap)
            sizes[k] = (uint32_t)n;
        ++k;
    });
    return k;
}

} // extern "C"

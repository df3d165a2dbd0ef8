// alac_common.h — device helpers shared by the ALAC encoder and decoder
// kernels (alac_encode.hip, alac_decode.hip): the reference's integer
// primitives (src/encoders/alac.c:907-1017, src/decoders/alac.c:1006-1145).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ALAC_MAX_ORDER 8 // MAX_LPC_ORDER (alac.c:25)
#define ALAC_SHIFT 2     // INTERLACING_SHIFT (alac.c:26)

// TRUNCATE_BITS (alac.c:918-930)
__device__ __forceinline__ int32_t alac_trunc(int32_t v, uint32_t bits)
{
    const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    const uint32_t t = (uint32_t)v & m;
    const uint32_t sb = bits >= 1 && bits <= 32 ? 1u << (bits - 1) : 0u;
    return (t & sb) ? (int32_t)(t - (m + 1u)) : (int32_t)t;
}

// SIGN_ONLY (alac.c:907-916)
__device__ __forceinline__ int32_t alac_sgn(int32_t v) { return (v > 0) - (v < 0); }

// floor(log2(v)) for v > 0 (the encoder's LOG2, alac.c:1007-1017)
__device__ __forceinline__ uint32_t alac_log2(uint32_t v) { return 31u - (uint32_t)__clz(v); }

// bits write_residual (alac.c:1081-1100) emits for `value` with parameter k
__device__ __forceinline__ uint32_t alac_code_bits(uint32_t value, uint32_t k, uint32_t ss)
{
    const uint32_t m = (1u << k) - 1u;
    if (value >= 9u * m) // MSB = value / m > 8: escape
        return 9u + ss;
    uint32_t msb = 0;
#pragma unroll
    for (uint32_t t = 1; t <= 8; ++t)
        msb += value >= t * m ? 1u : 0u;
    const uint32_t lsb = value - msb * m;
    return msb + 1u + (k > 1u ? (lsb > 0u ? k : k - 1u) : 0u);
}

// MSB-first bit reader over big-endian data held as 32-bit words (the image
// is 4-byte aligned and readable to a whole word past its end); reads past
// `end` return zeros and set `eof` (the reference longjmps: "EOF during
// frame reading").
struct ABitR {
    const uint32_t *w;
    uint64_t pos, end; // bit positions
    bool eof;
    __device__ __forceinline__ void init(const uint32_t *words, uint64_t bit0, uint64_t bit_end)
    {
        w = words;
        pos = bit0;
        end = bit_end;
        eof = false;
    }
    // the next 32 bits at pos (zeros past end are harmless: callers check eof)
    __device__ __forceinline__ uint32_t peek32() const
    {
        const uint64_t wi = pos >> 5;
        const uint32_t sh = (uint32_t)(pos & 31u);
        const uint32_t a = __builtin_bswap32(w[wi]);
        const uint32_t b = __builtin_bswap32(w[wi + 1]);
        return sh ? (a << sh) | (b >> (32u - sh)) : a;
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) // n <= 32
    {
        if (!n)
            return 0;
        if (pos + n > end) {
            eof = true;
            pos = end;
            return 0;
        }
        const uint32_t v = peek32() >> (32u - n);
        pos += n;
        return v;
    }
    __device__ __forceinline__ int32_t get_signed(uint32_t n)
    {
        const uint32_t v = get(n);
        if (n == 0 || n >= 32)
            return (int32_t)v;
        return (v & (1u << (n - 1))) ? (int32_t)(v - (1u << n)) : (int32_t)v;
    }
    // read_limited_unary(0, 9): 1-bits before a 0, at most 9 (-1 = 9 ones)
    __device__ __forceinline__ int32_t unary9()
    {
        const uint64_t avail = end > pos ? end - pos : 0;
        const uint32_t x = peek32();
        uint32_t ones = (uint32_t)__clz(~x); // leading ones (32 if all ones)
        if (ones >= 9) {
            if (avail < 9) {
                eof = true;
                pos = end;
                return 0;
            }
            pos += 9;
            return -1;
        }
        if (avail < ones + 1u) {
            eof = true;
            pos = end;
            return 0;
        }
        pos += ones + 1u;
        return (int32_t)ones;
    }
};

// The same reader for long sequential walks (residual blocks, frameset
// parses): the words under pos come from two 16-byte chunks held in
// registers (cur = chunk pos >> 7, nxt = the one after).  Entering the next
// chunk moves nxt to cur and issues the loads of the chunk after it, so a
// chunk's loads are in flight for the ~128 bits (several codes) before they
// are used -- ABitR waits for two dependent loads per code.  Loads are four
// dword loads (no alignment assumed) clamped to the last readable word
// (one whole word past `end`, as ABitR reads).
struct ABitRC {
    const uint32_t *w;
    uint64_t pos, end; // bit positions
    bool eof;
    uint64_t c, lim;   // chunk held in c0..c3; last readable word
    // (plain words, not a vector type: a dynamically indexed uint4 sends
    // the reader to LDS or scratch and every load is waited at once)
    uint32_t c0, c1, c2, c3, n0, n1, n2, n3;
    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return w[i < lim ? i : lim]; }
    __device__ __forceinline__ void load_next(uint64_t ch)
    {
        const uint64_t i = ch * 4u;
        if (i + 3u <= lim && (((uintptr_t)w & 15u) == 0u)) {
            // one 16-byte load: the lanes read 64 different streams, so
            // every vector load touches up to 64 cache lines -- four dword
            // loads cost four times the address work of one dwordx4
            const uint4 v = *(const uint4 *)(w + i);
            n0 = v.x;
            n1 = v.y;
            n2 = v.z;
            n3 = v.w;
        } else {
            n0 = ld(i);
            n1 = ld(i + 1);
            n2 = ld(i + 2);
            n3 = ld(i + 3);
        }
    }
    __device__ __forceinline__ void init(const uint32_t *words, uint64_t bit0, uint64_t bit_end)
    {
        w = words;
        pos = bit0;
        end = bit_end;
        eof = false;
        lim = (bit_end >> 5) + 1u;
        c = bit0 >> 7;
        load_next(c);
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
        load_next(c + 1u);
    }
    __device__ __forceinline__ uint32_t peek32()
    {
        const uint64_t pc = pos >> 7;
        if (pc != c) {
            if (pc != c + 1u) // a skip past the next chunk
                load_next(pc);
            c0 = n0;
            c1 = n1;
            c2 = n2;
            c3 = n3;
            load_next(pc + 1u);
            c = pc;
        }
        // word k and k + 1 of the eight by bit masks, not selects: a select
        // of two struct fields becomes a load through a selected address,
        // and the reader then lives in memory
        const uint32_t k = (uint32_t)(pos >> 5) & 3u;
        uint32_t m0 = 0u - (uint32_t)(k == 0u), m1 = 0u - (uint32_t)(k == 1u);
        uint32_t m2 = 0u - (uint32_t)(k == 2u), m3 = 0u - (uint32_t)(k == 3u);
        asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3));
        const uint32_t a = (c0 & m0) | (c1 & m1) | (c2 & m2) | (c3 & m3);
        const uint32_t b = (c1 & m0) | (c2 & m1) | (c3 & m2) | (n0 & m3);
        const uint32_t sh = (uint32_t)(pos & 31u);
        const uint32_t ha = __builtin_bswap32(a), hb = __builtin_bswap32(b);
        return sh ? (ha << sh) | (hb >> (32u - sh)) : ha;
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) // n <= 32
    {
        if (!n)
            return 0;
        if (pos + n > end) {
            eof = true;
            pos = end;
            return 0;
        }
        const uint32_t v = peek32() >> (32u - n);
        pos += n;
        return v;
    }
    __device__ __forceinline__ int32_t get_signed(uint32_t n)
    {
        const uint32_t v = get(n);
        if (n == 0 || n >= 32)
            return (int32_t)v;
        return (v & (1u << (n - 1))) ? (int32_t)(v - (1u << n)) : (int32_t)v;
    }
    __device__ __forceinline__ int32_t unary9()
    {
        const uint64_t avail = end > pos ? end - pos : 0;
        const uint32_t x = peek32();
        uint32_t ones = (uint32_t)__clz(~x);
        if (ones >= 9) {
            if (avail < 9) {
                eof = true;
                pos = end;
                return 0;
            }
            pos += 9;
            return -1;
        }
        if (avail < ones + 1u) {
            eof = true;
            pos = end;
            return 0;
        }
        pos += ones + 1u;
        return (int32_t)ones;
    }
};

// read_residual (decoders/alac.c:1087-1120): read_limited_unary(0, 9),
// then k bits of which an LSB field of 0 or 1 gives one back.  One peek
// covers both fields when they fit in 32 bits (ones <= 8 and k <= 23), with
// the reference's EOF order: the unary bits first, then all k bits
template <class R>
__device__ __forceinline__ uint32_t alac_read_residual(R &r, uint32_t k, uint32_t ss)
{
    const uint64_t avail = r.end > r.pos ? r.end - r.pos : 0;
    const uint32_t x = r.peek32();
    const uint32_t ones = (uint32_t)__clz(~x); // leading ones (32 if all ones)
    if (ones >= 9u) { // escape: a raw ss-bit value
        if (avail < 9u) {
            r.eof = true;
            r.pos = r.end;
            return 0;
        }
        r.pos += 9;
        return r.get(ss);
    }
    if (avail < ones + 1u || (k && avail < ones + 1u + k)) {
        r.eof = true;
        r.pos = r.end;
        return 0;
    }
    if (k == 0) {
        r.pos += ones + 1u;
        return ones;
    }
    const uint32_t m = (1u << k) - 1u;
    uint32_t lsb;
    if (ones + 1u + k <= 32u) {
        lsb = (x << (ones + 1u)) >> (32u - k);
    } else {
        r.pos += ones + 1u;
        lsb = r.peek32() >> (32u - k);
        r.pos -= ones + 1u;
    }
    if (lsb > 1u) {
        r.pos += ones + 1u + k;
        return ones * m + (lsb - 1u);
    }
    r.pos += ones + k; // ones + 1 + (k - 1)
    return ones * m;
}

// the decoder's LOG2 (decoders/alac.c:1006-1015): -1 for 0
__device__ __forceinline__ int32_t alac_log2s(int32_t v)
{
    return v == 0 ? -1 : (v < 0 ? 31 : 31 - (int32_t)__clz((uint32_t)v));
}

// read_residuals (decoders/alac.c:1017-1085) as a generator: next() yields
// the residuals one by one (zero runs expand inline); count() of produced
// residuals may reach residual_count + 1 (the reference's MIN bound)
struct AResidualReader {
    int32_t history;
    uint32_t sign_mod, hm, mk, ss, count;
    int32_t i;          // the reference's loop index
    uint32_t run_left;  // zeros still to hand out from a zero run
    __device__ void init(uint32_t residual_count, uint32_t sample_size, uint32_t initial_history,
                         uint32_t history_multiplier, uint32_t maximum_k)
    {
        history = (int32_t)initial_history;
        sign_mod = 0;
        hm = history_multiplier;
        mk = maximum_k;
        ss = sample_size;
        count = residual_count;
        i = 0;
        run_left = 0;
    }
    // next residual; false at the end or on EOF (r.eof)
    template <class R>
    __device__ __forceinline__ bool next(R &r, int32_t &out)
    {
        if (run_left) { // zeros of a zero block (the reference appends them
            --run_left; // inside the same loop iteration)
            out = 0;
            return true;
        }
        if (i >= (int32_t)count)
            return false;
        int32_t kk = alac_log2s((history >> 9) + 3);
        const uint32_t k = (uint32_t)kk < mk ? (uint32_t)kk : mk;
        const uint32_t u = alac_read_residual(r, k, ss) + sign_mod;
        if (r.eof)
            return false;
        sign_mod = 0;
        out = (u & 1u) ? -(int32_t)((u + 1u) >> 1) : (int32_t)(u >> 1);
        if (u > 0xFFFFu)
            history = 0xFFFF;
        else
            history = (int32_t)((uint32_t)history + (u * hm - (((uint32_t)history * hm) >> 9)));
        if (history < 128 && (i + 1) < (int32_t)count) {
            const int32_t lz = alac_log2s(history);
            const int32_t kz = 7 - lz + ((history + 16) / 64);
            const uint32_t k2 = (uint32_t)kz < mk ? (uint32_t)kz : mk;
            uint32_t z = alac_read_residual(r, k2, 16);
            if (r.eof)
                return false;
            if (z > 0) {
                const uint32_t cap = count - (uint32_t)i;
                z = z < cap ? z : cap;
                run_left = z;
                i += (int32_t)z;
            }
            history = 0;
            sign_mod = z <= 0xFFFFu ? 1u : 0u;
        }
        ++i;
        return true;
    }
};

// The residual walk's reader (k_adec_parse, ~24 k codes per lane and
// frameset): a 64-bit window W of the next bits, MSB first, topped up by a
// 32-bit word whenever fewer than 32 bits are left, the words taken in
// order from a 16-byte chunk in registers with the next chunk's load in
// flight (as ABitRC).  A code is one leading-ones count, one field
// extraction and a window shift, with no end-of-data test: the walk uses
// it only while at least 128 bits remain before `end` (two codes per
// residual step, 41 bits each at most), and hands the rest to the exact
// reader.
struct AFastBits {
    const uint32_t *w;
    uint64_t W;          // the next nb bits, MSB first
    uint32_t nb;         // valid bits in W (>= 32 between codes)
    uint64_t ci;         // chunk index of a0..a3
    uint32_t k;          // words of the chunk already in W
    uint64_t lim;        // last readable word (one past `end`, as ABitRC)
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3; // current and next chunk
    uint32_t used, room; // bits consumed since init; bits usable before the careful path

    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return w[i < lim ? i : lim]; }
    __device__ __forceinline__ void load_chunk(uint64_t ch)
    {
        const uint64_t i = ch * 4u;
        if (i + 3u <= lim && (((uintptr_t)w & 15u) == 0u)) {
            const uint4 v = *(const uint4 *)(w + i);
            b0 = v.x;
            b1 = v.y;
            b2 = v.z;
            b3 = v.w;
        } else {
            b0 = ld(i);
            b1 = ld(i + 1);
            b2 = ld(i + 2);
            b3 = ld(i + 3);
        }
    }
    // the next word in stream order, big-endian to host order
    __device__ __forceinline__ uint32_t next_word()
    {
        if (k == 4u) {
            a0 = b0;
            a1 = b1;
            a2 = b2;
            a3 = b3;
            ci += 1u;
            load_chunk(ci + 1u);
            k = 0u;
        }
        const uint32_t v = a0;
        a0 = a1;
        a1 = a2;
        a2 = a3;
        k += 1u;
        return __builtin_bswap32(v);
    }
    __device__ __forceinline__ void top_up()
    {
        if (nb < 32u) {
            W |= (uint64_t)next_word() << (32u - nb);
            nb += 32u;
        }
    }
    // top_up with selects: no divergent branch for the word itself, only
    // for a chunk change (every fourth word)
    __device__ __forceinline__ void top_up_sel()
    {
        if (k == 4u) { // the chunk is used up (next_word's lazy change)
            a0 = b0;
            a1 = b1;
            a2 = b2;
            a3 = b3;
            ci += 1u;
            load_chunk(ci + 1u);
            k = 0u;
        }
        const bool t = nb < 32u;
        const uint64_t wd = (uint64_t)__builtin_bswap32(a0);
        W |= t ? wd << ((32u - nb) & 63u) : 0ull;
        nb += t ? 32u : 0u;
        a0 = t ? a1 : a0;
        a1 = t ? a2 : a1;
        a2 = t ? a3 : a2;
        k += t ? 1u : 0u;
    }
    __device__ __forceinline__ void init(const uint32_t *words, uint64_t pos, uint64_t end)
    {
        w = words;
        lim = (end >> 5) + 1u;
        const uint64_t wi = pos >> 5;
        ci = wi >> 2;
        load_chunk(ci);
        a0 = b0;
        a1 = b1;
        a2 = b2;
        a3 = b3;
        load_chunk(ci + 1u);
        k = 0u;
        // skip to the word holding pos, then to its bit
        for (uint32_t s = (uint32_t)(wi & 3u); s > 0u; --s)
            next_word();
        W = (uint64_t)next_word() << 32;
        nb = 32u;
        top_up();
        const uint32_t sh = (uint32_t)(pos & 31u);
        W <<= sh;
        nb -= sh;
        top_up();
        used = 0u;
        const uint64_t avail = end > pos ? end - pos : 0u;
        room = avail > 128u + 0x7FFFFFFFull ? 0x7FFFFFFFu
                                            : (avail > 128u ? (uint32_t)(avail - 128u) : 0u);
    }
    __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(W >> 32); }
    __device__ __forceinline__ void skip(uint32_t n) // n <= 32
    {
        W <<= n;
        nb -= n;
        used += n;
        top_up();
    }
    // the next n bits (1 <= n <= 32)
    __device__ __forceinline__ uint32_t take(uint32_t n)
    {
        const uint32_t v = top32() >> (32u - n);
        skip(n);
        return v;
    }
    __device__ __forceinline__ bool careful() const { return used > room; }
    __device__ __forceinline__ void skip_sel(uint32_t n) // n <= 32
    {
        W <<= n;
        nb -= n;
        used += n;
        top_up_sel();
    }
};

// alac_read_residual on AFastBits, with at least 41 bits before `end`
// (no end-of-data case can arise)
__device__ __forceinline__ uint32_t alac_read_residual_fast(AFastBits &f, uint32_t k, uint32_t ss)
{
    const uint32_t x = f.top32();
    const uint32_t ones = (uint32_t)__clz(~x);
    if (ones >= 9u) { // escape: a raw ss-bit value
        f.skip(9u);
        return ss ? f.take(ss) : 0u;
    }
    if (k > 23u) { // ones + 1 + k may pass the 32 bits in view
        if (k == 0u) {
            f.skip(ones + 1u);
            return ones;
        }
        const uint32_t m = (1u << k) - 1u;
        f.skip(ones + 1u);
        const uint32_t lsb = f.top32() >> (32u - k);
        const bool big = lsb > 1u;
        f.skip(k - (big ? 0u : 1u));
        return ones * m + (big ? lsb - 1u : 0u);
    }
    // ones <= 8, k <= 23: both fields in x, no branch (k = 0: the unary
    // value alone)
    const uint32_t lsb = k ? (x << (ones + 1u)) >> ((32u - k) & 31u) : 0u;
    const uint32_t m = (1u << k) - 1u;
    const bool big = lsb > 1u;
    f.skip_sel(k ? ones + k + (big ? 1u : 0u) : ones + 1u);
    return k ? ones * m + (big ? lsb - 1u : 0u) : ones;
}

// AResidualReader::next on AFastBits (caller checked !f.careful())
__device__ __forceinline__ bool alac_next_fast(AResidualReader &g, AFastBits &f, int32_t &out)
{
    if (g.run_left) {
        --g.run_left;
        out = 0;
        return true;
    }
    if (g.i >= (int32_t)g.count)
        return false;
    const int32_t kk = alac_log2s((g.history >> 9) + 3);
    const uint32_t k = (uint32_t)kk < g.mk ? (uint32_t)kk : g.mk;
    const uint32_t u = alac_read_residual_fast(f, k, g.ss) + g.sign_mod;
    g.sign_mod = 0;
    out = (u & 1u) ? -(int32_t)((u + 1u) >> 1) : (int32_t)(u >> 1);
    if (u > 0xFFFFu)
        g.history = 0xFFFF;
    else
        g.history = (int32_t)((uint32_t)g.history + (u * g.hm - (((uint32_t)g.history * g.hm) >> 9)));
    if (g.history < 128 && (g.i + 1) < (int32_t)g.count) {
        const int32_t lz = alac_log2s(g.history);
        const int32_t kz = 7 - lz + ((g.history + 16) / 64);
        const uint32_t k2 = (uint32_t)kz < g.mk ? (uint32_t)kz : g.mk;
        uint32_t z = alac_read_residual_fast(f, k2, 16);
        if (z > 0) {
            const uint32_t cap = g.count - (uint32_t)g.i;
            z = z < cap ? z : cap;
            g.run_left = z;
            g.i += (int32_t)z;
        }
        g.history = 0;
        g.sign_mod = z <= 0xFFFFu ? 1u : 0u;
    }
    ++g.i;
    return true;
}

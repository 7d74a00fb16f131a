// gf256.hpp — host-side GF(2^8) arithmetic for the MI355X erasure-coding engine.
//
// Field: x^8 + x^4 + x^3 + x^2 + 1 (0x11D), generator 2 — the field ISA-L uses
// (ELECT's libec.so calls ISA-L at EC/erasure_coder.c:43, 57, 90, 128, 192, 221,
// 257, 274; EC/ = src/elect/src/native/src/org/apache/cassandra/io/erasurecode).
// Everything here is O(k^3) matrix work done once per coder or per erasure
// pattern; the byte-stream work is in rs_kernels.hip.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>

namespace elect {
namespace gf {

struct Field {
    std::array<uint8_t, 512> exp{};  // doubled so exp[a+b] needs no reduction
    std::array<uint8_t, 256> log{};
    constexpr Field()
    {
        unsigned v = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = static_cast<uint8_t>(v);
            log[v] = static_cast<uint8_t>(i);
            v <<= 1;
            if (v & 0x100u) v ^= 0x11Du;
        }
        exp[510] = exp[0];
        exp[511] = exp[1];
    }
};

inline constexpr Field kField{};

constexpr uint8_t mul(uint8_t a, uint8_t b)
{
    return (a == 0 || b == 0) ? 0 : kField.exp[kField.log[a] + kField.log[b]];
}

constexpr uint8_t inv(uint8_t a) { return a == 0 ? 0 : kField.exp[255 - kField.log[a]]; }

static_assert(mul(2, 0x80) == 0x1d, "0x11D reduction");
static_assert(inv(2) == 0x8e, "inverse of generator");

// Generator matrix used by ELECT (initEncodeMatrix, EC/erasure_coder.c:39-47):
// (k+m) x k, identity on top, Cauchy rows 1/(i^j) below.
inline void cauchy_generator(int k, int m, uint8_t* a)
{
    std::memset(a, 0, static_cast<size_t>(k + m) * k);
    for (int i = 0; i < k; ++i) a[i * k + i] = 1;
    for (int i = k; i < k + m; ++i)
        for (int j = 0; j < k; ++j) a[i * k + j] = inv(static_cast<uint8_t>(i ^ j));
}

// Gauss-Jordan inverse with the same pivot rule as the routine ELECT calls at
// EC/erasure_coder.c:257 (first lower row with a non-zero entry is swapped in).
// On a singular input it stops at the failing column and returns false with
// `out` partially reduced, which is what the reference then keeps using.
inline bool invert(uint8_t* work, uint8_t* out, int n)
{
    std::memset(out, 0, static_cast<size_t>(n) * n);
    for (int i = 0; i < n; ++i) out[i * n + i] = 1;
    for (int col = 0; col < n; ++col) {
        if (work[col * n + col] == 0) {
            int p = col + 1;
            for (; p < n; ++p)
                if (work[p * n + col] != 0) break;
            if (p == n) return false;
            for (int c = 0; c < n; ++c) {
                uint8_t t = work[col * n + c];
                work[col * n + c] = work[p * n + c];
                work[p * n + c] = t;
                t = out[col * n + c];
                out[col * n + c] = out[p * n + c];
                out[p * n + c] = t;
            }
        }
        const uint8_t s = inv(work[col * n + col]);
        for (int c = 0; c < n; ++c) {
            work[col * n + c] = mul(work[col * n + c], s);
            out[col * n + c] = mul(out[col * n + c], s);
        }
        for (int r = 0; r < n; ++r) {
            if (r == col) continue;
            const uint8_t f = work[r * n + col];
            if (f == 0) continue;  // x ^= 0*y is a no-op; skipping keeps results identical
            for (int c = 0; c < n; ++c) {
                out[r * n + c] ^= mul(f, out[col * n + c]);
                work[r * n + c] ^= mul(f, work[col * n + c]);
            }
        }
    }
    return true;
}

// ISA-L's 32-byte-per-coefficient table layout (ec_init_tables, called at
// EC/erasure_coder.c:57 and :192): c*x for x < 16, then c*(x<<4) for x < 16.
inline void isal_tables(const uint8_t* coef, int rows, int k, uint8_t* out)
{
    for (int e = 0; e < rows * k; ++e) {
        const uint8_t c = coef[e];
        for (int x = 0; x < 16; ++x) {
            out[32 * e + x] = mul(c, static_cast<uint8_t>(x));
            out[32 * e + 16 + x] = mul(c, static_cast<uint8_t>(x << 4));
        }
    }
}

// Byte-shuffle tables for the GPU kernel.  A byte x splits into bit fields
// x[2:0], x[5:3], x[7:6]; by linearity c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6].
// Each 8-entry table is two dwords (entries 0-3 in `lo`, 4-7 in `hi`) so one
// v_perm_b32 looks up four bytes at once; T2 has 4 entries in one dword.
struct PermTable {
    uint32_t t0_lo, t0_hi, t1_lo, t1_hi, t2;
};

inline PermTable perm_table(uint8_t c)
{
    uint8_t t0[8], t1[8], t2[4];
    for (int i = 0; i < 8; ++i) {
        t0[i] = mul(c, static_cast<uint8_t>(i));
        t1[i] = mul(c, static_cast<uint8_t>(i << 3));
    }
    for (int i = 0; i < 4; ++i) t2[i] = mul(c, static_cast<uint8_t>(i << 6));
    auto pack = [](const uint8_t* b) {
        return static_cast<uint32_t>(b[0]) | static_cast<uint32_t>(b[1]) << 8 |
               static_cast<uint32_t>(b[2]) << 16 | static_cast<uint32_t>(b[3]) << 24;
    };
    return PermTable{pack(t0), pack(t0 + 4), pack(t1), pack(t1 + 4), pack(t2)};
}

}  // namespace gf
}  // namespace elect

// pargz.cpp -- single-stream gzip input inflated on several threads (see pargz.h).
//
// Deflate (RFC 1951) decoding is written here from the format: a 64-bit LSB-first bit buffer,
// two-level Huffman tables (11 primary bits for literal/length codes, 10 for distances), and the
// validity rules of zlib's inflate (over-subscribed codes, incomplete codes other than a single
// length-1 code, a missing end-of-block code, bit-length repeats past the end, distances further
// back than the history), so a stream this decoder accepts is one zlib accepts up to the same byte.
#include "pargz.h"

#include <dlfcn.h>
#include <emmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace fqhost {
namespace {

constexpr uint32_t kWin = 32768;  // deflate's history
#ifndef FQ_PARGZ_LITBITS
#define FQ_PARGZ_LITBITS 11  // primary literal/length table bits (profiling: tools/pargz_ab.py)
#endif
#ifndef FQ_PARGZ_TWOLIT
#define FQ_PARGZ_TWOLIT 1  // two literals per primary entry where both codes fit (profiling: 0)
#endif
#ifndef FQ_PARGZ_DISTBITS
#define FQ_PARGZ_DISTBITS 8  // (8 vs 10 bits: medians -2 to +8 % over two passes, inside the run-to-run spread; kept, a smaller table to build per block; profiles/r06_pargz_ab.txt)
#endif
constexpr int kLitBits = FQ_PARGZ_LITBITS, kDistBits = FQ_PARGZ_DISTBITS, kClBits = 7;

// ---- bit reader (LSB first; reads past the end as zero bits, overrun() tells) ----
struct Bits {
    const uint8_t* p = nullptr;
    size_t n = 0, pos = 0;  // pos: next byte to load
    uint64_t buf = 0;
    int cnt = 0;
    void seek(const uint8_t* data, size_t len, uint64_t bit) {
        p = data;
        n = len;
        pos = (size_t)(bit >> 3);
        buf = 0;
        cnt = 0;
        refill();
        consume((int)(bit & 7));
    }
    void refill() {  // cnt >= 56 afterwards (the bits above cnt are the following input bits)
        if (pos + 8 <= n) {
            uint64_t v;
            std::memcpy(&v, p + pos, 8);
            buf |= v << cnt;
            pos += (size_t)((63 - cnt) >> 3);
            cnt |= 56;
        } else {
            while (cnt <= 56) {
                buf |= (uint64_t)(pos < n ? p[pos] : 0) << cnt;
                ++pos;
                cnt += 8;
            }
        }
    }
    uint64_t bitpos() const { return (uint64_t)pos * 8 - (uint64_t)cnt; }
    bool overrun() const { return bitpos() > (uint64_t)n * 8; }
    void consume(int k) {
        buf >>= k;
        cnt -= k;
    }
    uint32_t get(int k) {  // k <= 32
        if (cnt < k) refill();
        const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1));
        consume(k);
        return v;
    }
};

// ---- Huffman tables ----
// entry: bits 0-4 code length (0: no such code), bit 5 subtable pointer, bits 8-11 subtable bits,
// bits 16-31 the symbol (code-length codes), or the subtable offset.  Literal/length and distance
// tables carry the decoded value instead, so the decode loop needs no second lookup:
//   literal/length: bit 7 literal (bits 16-23 the byte), bit 6 length (bits 16-24 the base
//     length, bits 12-15 its extra bits); neither: end of block when bits 16-31 are 256, else an
//     invalid symbol (286, 287);
//   distance: bit 7 valid (bits 16-31 the base distance, bits 12-15 its extra bits); not valid:
//     symbols 30, 31.
struct Table {
    std::vector<uint32_t> e;
    int pbits = 0;
};
enum Kind { kCodes, kLens, kDists };
constexpr uint32_t kSub = 32, kLit = 128, kLen = 64, kDistOk = 128;

uint32_t rev_bits(uint32_t c, int len) {
    uint32_t r = 0;
    for (int i = 0; i < len; ++i) r |= ((c >> i) & 1u) << (len - 1 - i);
    return r;
}

const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// the entry bits above the code length for symbol s of a table of this kind
uint32_t entry_value(int s, Kind kind) {
    if (kind == kLens) {
        if (s < 256) return (uint32_t)s << 16 | kLit;
        if (s >= 257 && s <= 285) return (uint32_t)kLenBase[s - 257] << 16 | (uint32_t)kLenExtra[s - 257] << 12 | kLen;
        return (uint32_t)s << 16;  // 256: end of block; 286, 287: invalid
    }
    if (kind == kDists) return s < 30 ? (uint32_t)kDistBase[s] << 16 | (uint32_t)kDistExtra[s] << 12 | kDistOk : 0u;
    return (uint32_t)s << 16;
}

// zlib's inflate_table rules: over-subscribed -> invalid; incomplete -> invalid unless the code
// lengths are lit/len or distance codes whose longest code has length 1; no codes at all -> a table
// whose every entry is invalid
bool build(Table& t, const uint8_t* lens, int n, int pbits, Kind kind) {
    int count[16] = {0};
    for (int i = 0; i < n; ++i) ++count[lens[i]];
    int mx = 15;
    while (mx >= 1 && count[mx] == 0) --mx;
    t.pbits = pbits;
    t.e.assign((size_t)1 << pbits, 0u);
    if (mx == 0) return true;
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return false;
    }
    if (left > 0 && (kind == kCodes || mx != 1)) return false;
    uint32_t next[16];
    uint32_t code = 0;
    count[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + (uint32_t)count[l - 1]) << 1;
        next[l] = code;
    }
    const int sbits = std::max(0, mx - pbits);
    thread_local std::vector<int> sub;  // (per-thread scratch: the block-start search builds many tables)
    sub.assign((size_t)1 << pbits, -1);
    for (int s = 0; s < n; ++s) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t r = rev_bits(next[l]++, l);
        const uint32_t v = entry_value(s, kind) | (uint32_t)l;
        if (l <= pbits) {
            for (uint32_t k = r; k < (1u << pbits); k += 1u << l) t.e[k] = v;
        } else {
            const uint32_t pre = r & ((1u << pbits) - 1);
            int& off = sub[pre];
            if (off < 0) {
                off = (int)t.e.size();
                t.e.resize(t.e.size() + ((size_t)1 << sbits), 0u);
                t.e[pre] = (uint32_t)off << 16 | (uint32_t)sbits << 8 | kSub;
            }
            for (uint32_t k = r >> pbits; k < (1u << sbits); k += 1u << (l - pbits)) t.e[(size_t)off + k] = v;
        }
    }
    if (FQ_PARGZ_TWOLIT && kind == kLens) {
        // two literals in one primary entry where the second code also lies in the primary bits
        // (bits 24-31 the second byte, bit 8 set, bits 0-4 both code lengths): literal-heavy text
        // (FASTQ bases and qualities, codes of 2-6 bits) decodes two symbols per lookup
        const uint32_t full = 1u << pbits;
        thread_local std::vector<uint32_t> one;
        one.assign(t.e.begin(), t.e.begin() + full);
        for (uint32_t i = 0; i < full; ++i) {
            const uint32_t e = one[i];
            if (!(e & kLit)) continue;
            const int l1 = (int)(e & 31);
            const uint32_t e2 = one[i >> l1];
            if ((e2 & kLit) && (int)(e2 & 31) <= pbits - l1)
                t.e[i] = (e & 0x00ff0000u) | ((e2 >> 16) & 255u) << 24 | 256u | kLit | (uint32_t)(l1 + (int)(e2 & 31));
        }
    }
    return true;
}

// the entry of the next code (the bit buffer must hold >= 15 bits)
inline uint32_t lookup(const Table& t, uint64_t buf) {
    uint32_t e = t.e[buf & ((1u << t.pbits) - 1)];
    if (e & kSub) e = t.e[(e >> 16) + ((buf >> t.pbits) & ((1u << ((e >> 8) & 15)) - 1))];
    return e;
}

struct Fixed {
    Table lit, dist;
    Fixed() {
        uint8_t l[288], d[32];
        for (int i = 0; i < 288; ++i) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
        for (int i = 0; i < 32; ++i) d[i] = 5;
        build(lit, l, 288, kLitBits, kLens);
        build(dist, d, 32, kDistBits, kDists);  // (symbols 30 and 31 decode, then fail: "invalid distance code")
    }
};
const Fixed& fixed_tables() {
    static const Fixed f;
    return f;
}

// growable array of T without value-initialisation (the decoder writes every element it keeps)
template <class T>
struct PodBuf {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    PodBuf() = default;
    PodBuf(const PodBuf&) = delete;
    PodBuf& operator=(const PodBuf&) = delete;
    PodBuf(PodBuf&& o) noexcept { *this = std::move(o); }
    PodBuf& operator=(PodBuf&& o) noexcept {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(cap, o.cap);
        return *this;
    }
    ~PodBuf() { std::free(p); }
    void reserve(size_t c) {
        if (c <= cap) return;
        c = std::max(c, cap + cap / 2);
        T* q = static_cast<T*>(std::realloc(p, c * sizeof(T)));
        if (!q) throw std::bad_alloc();
        p = q;
        cap = c;
    }
    void assign(const T* src, size_t k) {
        n = 0;
        reserve(k);
        if (k) std::memcpy(p, src, k * sizeof(T));
        n = k;
    }
    void release() {
        std::free(p);
        p = nullptr;
        n = cap = 0;
    }
    size_t size() const { return n; }
    T* data() { return p; }
    const T* data() const { return p; }
};

// ---- output ----
// Bytes with the history in front (win bytes of the stream before them), or 16-bit symbols where
// 256 + i stands for byte i of the unknown 32 KiB before the output.
struct Out8 {
    PodBuf<uint8_t> b;
    size_t win = 0;  // history bytes at the front
};
struct Out16 {
    PodBuf<uint16_t> s;
    // no marker among the last 32 KiB of symbols (scanned backwards: on FASTQ one turns up within a
    // few symbols, so the test costs next to nothing while markers persist)
    bool tail_clean() const {
        if (s.n < kWin) return false;
        const uint16_t* e = s.p + s.n;
        const __m128i z = _mm_setzero_si128();
        for (size_t k = 8; k <= kWin; k += 8) {
            const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(e - k));
            if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_srli_epi16(x, 8), z)) != 0xffff) return false;
        }
        return true;
    }
};

enum Status { kBlockDone, kFinalDone, kError };

struct Decoder {
    Table cl, lit, dist;
    // output cap of the code loop (symbols in the buffer): reaching it is an error, so a chunk that
    // expands far beyond FASTQ's ratios (a run of one byte, say) sends the file to zlib's reader
    // instead of holding gigabytes per chunk in flight
    size_t max_sym = SIZE_MAX;
    uint8_t lens[320];

    // a dynamic block's header -> lit / dist tables
    bool dynamic_header(Bits& br) {
        br.refill();
        const int hlit = (int)br.get(5) + 257, hdist = (int)br.get(5) + 1, hclen = (int)br.get(4) + 4;
        if (hlit > 286 || hdist > 30) return false;
        static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        uint8_t cll[19] = {0};
        for (int i = 0; i < hclen; ++i) cll[order[i]] = (uint8_t)br.get(3);
        if (!build(cl, cll, 19, kClBits, kCodes)) return false;
        int n = 0;
        const int total = hlit + hdist;
        while (n < total) {
            if (br.cnt < 16) br.refill();
            const uint32_t e = lookup(cl, br.buf);
            const int l = (int)(e & 31);
            if (!l) return false;
            br.consume(l);
            const int sym = (int)(e >> 16);
            if (sym < 16) {
                lens[n++] = (uint8_t)sym;
                continue;
            }
            int rep, val = 0;
            if (sym == 16) {
                if (n == 0) return false;
                val = lens[n - 1];
                rep = 3 + (int)br.get(2);
            } else if (sym == 17) {
                rep = 3 + (int)br.get(3);
            } else {
                rep = 11 + (int)br.get(7);
            }
            if (n + rep > total) return false;
            while (rep--) lens[n++] = (uint8_t)val;
        }
        if (br.overrun()) return false;
        if (lens[256] == 0) return false;
        return build(lit, lens, hlit, kLitBits, kLens) && build(dist, lens + hlit, hdist, kDistBits, kDists);
    }

    // one block into o (8-bit output with history, or 16-bit symbols with markers)
    template <class O>
    Status block(Bits& br, O& o) {
        br.refill();
        const bool final_ = br.get(1) != 0;
        const uint32_t type = br.get(2);
        const Table* lt;
        const Table* dt;
        if (type == 0) {  // stored
            br.consume(br.cnt & 7);  // (to the byte boundary)
            const uint32_t len = br.get(16), nlen = br.get(16);
            if ((len ^ 0xffffu) != nlen) return kError;
            // the rest of the bit buffer holds whole bytes; take them first, then the input
            uint32_t left = len;
            while (left && br.cnt >= 8) {
                put_byte(o, (uint8_t)(br.buf & 0xff));
                br.consume(8);
                --left;
            }
            const uint64_t at = br.bitpos() >> 3;
            if (at + left > br.n) return kError;
            for (uint32_t i = 0; i < left; ++i) put_byte(o, br.p[at + i]);
            br.seek(br.p, br.n, (at + left) * 8);
            return final_ ? kFinalDone : kBlockDone;
        } else if (type == 1) {
            lt = &fixed_tables().lit;
            dt = &fixed_tables().dist;
        } else if (type == 2) {
            if (!dynamic_header(br)) return kError;
            lt = &lit;
            dt = &dist;
        } else {
            return kError;
        }
        if (!codes(br, o, *lt, *dt)) return kError;
        return final_ ? kFinalDone : kBlockDone;
    }

    static void put_byte(Out8& o, uint8_t v) {
        o.b.reserve(o.b.n + 1);
        o.b.p[o.b.n++] = v;
    }
    static void put_byte(Out16& o, uint8_t v) {
        o.s.reserve(o.s.n + 1);
        o.s.p[o.s.n++] = v;
    }

    // one block's codes.  The bit buffer, the tables and the output live in locals (byte stores
    // alias everything: members would be reloaded after each one); >= 48 bits are in the buffer at
    // each code, enough for a length, its extra bits, a distance and its extra bits.
    template <class T, bool kSym>
    static bool codes_impl(Bits& br, PodBuf<T>& v, const Table& lt, const Table& dt, size_t stop_at = SIZE_MAX,
                           bool* paused = nullptr) {
        const uint32_t* __restrict L = lt.e.data();
        const uint32_t* __restrict D = dt.e.data();
        const int lb = lt.pbits, db = dt.pbits;
        const uint64_t lm = (1ull << lb) - 1, dm = (1ull << db) - 1;
        const uint8_t* __restrict in = br.p;
        const size_t n = br.n;
        uint64_t buf = br.buf;
        int cnt = br.cnt;
        size_t pos = br.pos;
        size_t sz = v.n;
        v.reserve(sz + 65536);
        T* __restrict b = v.p;
        size_t cap = v.cap;
        size_t lim = std::min(cap - 300, stop_at);  // (the output's room, or where to pause)
        bool ok = false;
        for (;;) {
            if (cnt < 48) {
                if (pos + 8 <= n) {
                    uint64_t w;
                    std::memcpy(&w, in + pos, 8);
                    buf |= w << cnt;
                    pos += (size_t)((63 - cnt) >> 3);
                    cnt |= 56;
                } else {
                    while (cnt <= 56) {
                        buf |= (uint64_t)(pos < n ? in[pos] : 0) << cnt;
                        ++pos;
                        cnt += 8;
                    }
                    if (pos > n + 8) break;  // (past the input: truncated, or a false start)
                }
            }
            if (sz >= lim) {
                if (sz >= stop_at) {  // (paused at a code boundary: a later call goes on from here)
                    *paused = true;
                    break;
                }
                v.n = sz;
                v.reserve(cap * 2);
                b = v.p;
                cap = v.cap;
                lim = std::min(cap - 300, stop_at);
            }
            uint32_t e = L[buf & lm];
            if (e & kSub) e = L[(e >> 16) + ((buf >> lb) & ((1u << ((e >> 8) & 15)) - 1))];
            const int l = (int)(e & 31);
            if (e & kLit) {  // one or two literals (the second store is past the end when one)
                buf >>= l;
                cnt -= l;
                b[sz] = (T)((e >> 16) & 255);
                b[sz + 1] = (T)(e >> 24);
                sz += 1 + ((e >> 8) & 1);
                continue;
            }
            if (!(e & kLen)) {  // end of block, or an invalid code / symbol
                if (l && (e >> 16) == 256) {
                    buf >>= l;
                    cnt -= l;
                    ok = (uint64_t)pos * 8 - (uint64_t)cnt <= (uint64_t)n * 8;
                }
                break;
            }
            buf >>= l;
            cnt -= l;
            const int xl = (int)((e >> 12) & 15);
            const uint32_t len = (e >> 16) + (uint32_t)(buf & ((1ull << xl) - 1));
            buf >>= xl;
            cnt -= xl;
            uint32_t d = D[buf & dm];
            if (d & kSub) d = D[(d >> 16) + ((buf >> db) & ((1u << ((d >> 8) & 15)) - 1))];
            if (!(d & kDistOk)) break;
            const int dl = (int)(d & 31);
            buf >>= dl;
            cnt -= dl;
            const int xd = (int)((d >> 12) & 15);
            const uint32_t dist = (d >> 16) + (uint32_t)(buf & ((1ull << xd) - 1));
            buf >>= xd;
            cnt -= xd;
            T* dst = b + sz;
            if (!kSym) {
                if (dist > sz) break;  // further back than the history
                const T* src = dst - dist;
                if (dist >= 32) {  // 32 bytes at once, then 16 a step (up to 31 past the length: cap has room)
                    std::memcpy(dst, src, 16);
                    std::memcpy(dst + 16, src + 16, 16);
                    for (uint32_t i = 32; i < len; i += 16) std::memcpy(dst + i, src + i, 16);
                } else if (dist >= 16) {  // 16 bytes a step (may write up to 15 past the length: cap has room)
                    for (uint32_t i = 0; i < len; i += 16) std::memcpy(dst + i, src + i, 16);
                } else if (dist >= 8) {
                    for (uint32_t i = 0; i < len; i += 8) std::memcpy(dst + i, src + i, 8);
                } else if (dist == 1) {
                    std::memset(dst, (int)src[0], len);
                } else {
                    for (uint32_t i = 0; i < len; ++i) dst[i] = src[i];
                }
            } else {
                if (dist > sz + kWin) break;  // (beyond any window)
                // (markers are not tracked here: decode_from looks for one in the last 32 KiB at
                // each block end, where on FASTQ a backward scan meets one within a few symbols)
                if (dist <= sz) {  // within the chunk's own output
                    const T* src = dst - dist;
                    if (dist >= 16) {  // 16 symbols a step (most matches: FASTQ's are ~10 long; may
                                       // write up to 15 past the length: cap has room)
                        for (uint32_t i = 0; i < len; i += 16) {
                            const __m128i x0 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
                            const __m128i x1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 8));
                            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i), x0);
                            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 8), x1);
                        }
                    } else if (dist >= 8) {  // 8 symbols a step (each step's source written before it)
                        for (uint32_t i = 0; i < len; i += 8)
                            _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i),
                                             _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i)));
                    } else if (dist == 1) {
                        const T x = src[0];
                        for (uint32_t i = 0; i < len; ++i) dst[i] = x;
                    } else {
                        for (uint32_t i = 0; i < len; ++i) dst[i] = src[i];
                    }
                } else {  // (partly) the unknown history: markers 256 + its index
                    for (uint32_t i = 0; i < len; ++i) {
                        const int64_t s = (int64_t)sz + i - (int64_t)dist;
                        dst[i] = s >= 0 ? b[(size_t)s] : (T)(256 + kWin + s);
                    }
                }
            }
            sz += len;
        }
        br.buf = buf;
        br.cnt = cnt;
        br.pos = pos;
        v.n = sz;
        return ok;
    }

    bool codes(Bits& br, Out8& o, const Table& lt, const Table& dt) {
        bool capped = false;
        return codes_impl<uint8_t, false>(br, o.b, lt, dt, max_sym, &capped) && !capped;
    }
    bool codes(Bits& br, Out16& o, const Table& lt, const Table& dt) {
        bool capped = false;
        return codes_impl<uint16_t, true>(br, o.s, lt, dt, max_sym, &capped) && !capped;
    }
};

// ---- gzip header ----
// offset of the deflate data of the member at `o`, or 0 when it is not a gzip member header
size_t member_data(const uint8_t* p, size_t n, size_t o) {
    if (n - o < 18 || p[o] != 0x1f || p[o + 1] != 0x8b || p[o + 2] != 8 || (p[o + 3] & 0xe0)) return 0;
    const uint8_t flg = p[o + 3];
    size_t q = o + 10;
    if (flg & 4) {
        if (q + 2 > n) return 0;
        q += 2 + ((size_t)p[q] | (size_t)p[q + 1] << 8);
    }
    for (int f : {8, 16})
        if (flg & f) {
            while (q < n && p[q]) ++q;
            ++q;
        }
    if (flg & 2) q += 2;
    return q < n ? q : 0;
}

uint32_t (*crc_fn())(uint32_t, const void*, size_t) {
    static uint32_t (*f)(uint32_t, const void*, size_t) = [] {
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        return h ? reinterpret_cast<uint32_t (*)(uint32_t, const void*, size_t)>(dlsym(h, "libdeflate_crc32")) : nullptr;
    }();
    return f;
}
// CRC32 of n more bytes after `c` (the CRC of what came before them; 0 at the start)
uint32_t crc_more(uint32_t c, const uint8_t* p, size_t n) {
    if (auto f = crc_fn()) return f(c, p, n);
    for (size_t o = 0; o < n; o += (size_t)1 << 30) c = (uint32_t)crc32(c, p + o, (uInt)std::min(n - o, (size_t)1 << 30));
    return c;
}
uint32_t crc_of(const uint8_t* p, size_t n) { return crc_more(0, p, n); }

// Kraft sums (128 >> l per nonzero length l) of four three-bit code lengths, by their 12 bits
const uint16_t* kraft4() {
    static const std::vector<uint16_t> t = [] {
        std::vector<uint16_t> v(4096);
        for (int i = 0; i < 4096; ++i) {
            int s = 0;
            for (int k = 0; k < 4; ++k) {
                const int l = (i >> (3 * k)) & 7;
                if (l) s += 128 >> l;
            }
            v[(size_t)i] = (uint16_t)s;
        }
        return v;
    }();
    return t.data();
}

}  // namespace

// ---- the chunked source ----
struct ParGzSource::Impl {
    struct Chunk {
        uint64_t nom0 = 0, nom1 = 0;  // nominal range of block starts [nom0, nom1) (bits)
        // the worker's decode
        int64_t start = -1;  // bit where it started (-1: no block start found in range)
        uint64_t end = 0;    // bit after its last block
        bool final_ = false, error = false;
        Out16 o16;           // speculative prefix (markers)
        Out8 o8;             // bytes (after the prefix; o8.win history bytes in front)
        // after resolution
        PodBuf<uint8_t> pre;       // the prefix resolved
        uint32_t crc = 0;
        size_t bytes = 0;
        std::vector<uint8_t> window;  // the stream's last <= 32 KiB through this chunk
        bool decoded = false, windowed = false, ready = false;
        bool beyond = false;  // after the final block: not part of the stream
    };
    const uint8_t* map = nullptr;
    size_t size = 0;
    size_t data0 = 0;  // deflate data start (bytes)
    size_t call = 1 << 20;
    std::string path;
    std::vector<Chunk> ch;
    std::mutex m;
    std::condition_variable cv;
    size_t next_take = 0;      // next chunk a worker takes
    size_t consumed = 0;       // chunks handed out completely (freed)
    size_t ahead = 8;          // chunks decoded ahead of the consumer
    std::atomic<bool> stop{false};
    bool anomaly = false;      // the parallel path gives up: zlib from the start
    std::vector<std::thread> th;
    // consumer
    size_t cur = 0, cur_pos = 0;  // chunk being handed out, bytes of it handed out
    uint64_t handed = 0, good = 0;  // stream bytes handed out; through the ready chunks
    bool finished = false;        // the member's final block and trailer verified, EOF after it
    uint32_t crc_all = 0;
    // fallback: zlib's stream reader from the start, the handed-out bytes skipped
    gzFile gz = nullptr;
    bool fb = false, fb_bad = false, fb_end = false, reported = false;
    std::vector<char> fb_buf;
    size_t fb_off = 0;

    // output buffers go back to a pool when a chunk is done with them: the next chunk writes into
    // pages already mapped (fresh tens of MiB per chunk cost more in page faults than the decode)
    std::mutex pool_m;
    std::vector<PodBuf<uint8_t>> pool8;
    std::vector<PodBuf<uint16_t>> pool16;
    template <class T>
    std::vector<PodBuf<T>>& pool_of();
    template <class T>
    void take(PodBuf<T>& b) {
        std::lock_guard<std::mutex> g(pool_m);
        auto& pl = pool_of<T>();
        if (b.cap || pl.empty()) return;
        b = std::move(pl.back());
        pl.pop_back();
        b.n = 0;
    }
    template <class T>
    void give(PodBuf<T>& b) {
        if (!b.cap) return;
        b.n = 0;
        std::lock_guard<std::mutex> g(pool_m);
        pool_of<T>().push_back(std::move(b));
    }

    std::atomic<uint64_t> n_redecode{0}, n_nostart{0}, n_beyond{0}, find_ns{0}, cand_tried{0}, dec_ns{0}, res_ns{0}, sym16_n{0}, crc_ns{0}, wait_ns{0};
    ~Impl() {
        if (std::getenv("FQ_PARGZ_DEBUG"))
            fprintf(stderr, "pargz: %zu chunks, %llu without a start, %llu decoded again, %llu beyond the end, %llu candidates tried, find %.3f s, decode %.3f s, resolve %.3f s (waiting %.3f s, crc %.3f s), %llu symbols with markers\n",
                    ch.size(), (unsigned long long)n_nostart.load(), (unsigned long long)n_redecode.load(),
                    (unsigned long long)n_beyond.load(), (unsigned long long)cand_tried.load(), find_ns.load() * 1e-9,
                    dec_ns.load() * 1e-9, res_ns.load() * 1e-9, wait_ns.load() * 1e-9, crc_ns.load() * 1e-9, (unsigned long long)sym16_n.load());
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
        if (gz) gzclose(gz);
        if (map) munmap(const_cast<uint8_t*>(map), size);
    }

    // ---- worker side ----
    // the first bit offset in [from, to) where a dynamic block starts that decodes as one (16-bit
    // symbols, so references before it are markers); its output in c.o16
    bool find_start(Chunk& c, Decoder& dec) {
        Bits br;
        const uint64_t lim = std::min<uint64_t>(c.nom1, (uint64_t)size * 8);
        uint64_t cand = 0, base = 0;  // bit i of cand: offset base + i passes the header checks
        bool have = false;
        for (uint64_t b = c.nom0; b < lim; ++b) {
            // quick rejects on the header bits, 64 offsets at a time: BFINAL 0, BTYPE 2 (bits 001),
            // HLIT <= 29 and HDIST <= 29 (their top four bits not all set)
            if (!have || b >= base + 64) {
                base = b;
                const size_t by = (size_t)(b >> 3);
                if (by + 24 > size) return false;
                unsigned __int128 x;
                std::memcpy(&x, map + by, 16);
                x >>= (b & 7);  // (121 valid bits: the 64 offsets' first 13 bits)
                cand = (uint64_t)(~x & ~(x >> 1) & (x >> 2) & ~((x >> 4) & (x >> 5) & (x >> 6) & (x >> 7)) &
                                  ~((x >> 9) & (x >> 10) & (x >> 11) & (x >> 12)));
                have = true;
            }
            const uint64_t m = cand >> (b - base);
            if (!m) {  // (none left in this window: the next one starts at base + 64)
                b = base + 63;
                have = false;
                continue;
            }
            b += (uint64_t)__builtin_ctzll(m);
            if (b >= lim) return false;
            // the code-length code (HCLEN + 4 three-bit lengths from bit 17) must be complete:
            // Kraft sum of its lengths (128 >> l each) exactly 128, four lengths per table lookup
            {
                const uint64_t c17 = b + 17;
                if ((c17 >> 3) + 8 > size) return false;
                uint64_t v;
                std::memcpy(&v, map + (c17 >> 3), 8);
                v >>= (c17 & 7);
                uint64_t hw;
                std::memcpy(&hw, map + (b >> 3), 8);
                const int ncl = (int)((hw >> (b & 7) >> 13) & 15) + 4;
                const uint16_t* kr = kraft4();
                const uint64_t vv = v & ((1ull << (3 * ncl)) - 1);  // (3 ncl <= 57)
                const uint32_t sum = kr[vv & 4095] + kr[(vv >> 12) & 4095] + kr[(vv >> 24) & 4095] + kr[(vv >> 36) & 4095] +
                                     kr[(vv >> 48) & 4095];
                if (sum != 128) continue;
            }
            br.seek(map, size, b);
            if (stop) return false;
            ++cand_tried;
            take(c.o16.s);
            c.o16.s.n = 0;
            // (a false start can decode as a block: its literals are then random bytes.  FASTQ is
            // text, so a block whose literals are not is passed over -- only a speed matter: the
            // start of every chunk is verified against the previous chunk's end.  With complete
            // codes every bit pattern decodes, so a false start may run on for many kilobytes until
            // it happens on an end-of-block code: its first 1024 symbols are judged first.)
            auto implausible = [&](size_t n) {
                size_t odd = 0;
                for (size_t k = 0; k < n; ++k) {
                    const uint16_t x = c.o16.s.p[k];
                    odd += x < 256 && x != '\n' && x != '\r' && x != '\t' && (x < 32 || x > 126);
                }
                return odd * 200 > n;
            };
            br.refill();
            br.consume(3);  // (BFINAL 0, BTYPE 2: checked above)
            if (!dec.dynamic_header(br)) continue;
            bool paused = false;
            bool ok = Decoder::codes_impl<uint16_t, true>(br, c.o16.s, dec.lit, dec.dist, 1024, &paused);
            if (paused) {
                if (implausible(c.o16.s.n)) continue;
                paused = false;
                ok = Decoder::codes_impl<uint16_t, true>(br, c.o16.s, dec.lit, dec.dist, dec.max_sym, &paused) && !paused;
            }
            if (!ok || implausible(c.o16.s.n) || c.o16.s.n < 64) continue;
            const Status st = kBlockDone;
            c.start = (int64_t)b;
            c.end = br.bitpos();
            c.final_ = st == kFinalDone;
            return true;
        }
        return false;
    }

    // decode blocks from br until a block ends at or past c.nom1 (or the final block); 16-bit
    // symbols until the last 32 KiB hold no marker, then bytes
    void decode_from(Chunk& c, Bits& br, Decoder& dec, bool sym16) {
        for (;;) {
            if (c.final_ || br.bitpos() >= c.nom1) break;
            if (sym16 && c.o16.tail_clean()) {
                // no marker can appear any more: the rest as bytes, the last 32 KiB as history
                const size_t k = c.o16.s.n;
                take(c.o8.b);
                c.o8.b.reserve(kWin);
                for (size_t i = 0; i < kWin; ++i) c.o8.b.p[i] = (uint8_t)c.o16.s.p[k - kWin + i];
                c.o8.b.n = kWin;
                c.o8.win = kWin;
                sym16 = false;
            }
            const Status st = sym16 ? dec.block(br, c.o16) : dec.block(br, c.o8);
            if (st == kError) {
                c.error = true;
                break;
            }
            c.end = br.bitpos();
            if (st == kFinalDone) c.final_ = true;
        }
    }

    void work() {
        Decoder dec;
        for (;;) {
            size_t i;
            {
                std::unique_lock<std::mutex> lk(m);
                // (ahead of the consumer's verified frontier, not of what it handed out: bytes go out
                // in whole gzread calls, which may span more chunks than `ahead`)
                cv.wait(lk, [&] { return stop || next_take >= ch.size() || next_take < next_good + ahead; });
                if (stop || next_take >= ch.size()) return;
                i = next_take++;
            }
            Chunk& c = ch[i];
            Bits br;
            // (16 times the chunk's compressed bytes, FASTQ inflating 3-6 times, and at least 16 MiB:
            // a chunk's decode runs on to the end of the block that crosses its end)
            dec.max_sym = std::max<size_t>((size_t)((c.nom1 - c.nom0) >> 3) * 16, (size_t)16 << 20) + ((size_t)1 << 16);
            const auto d0 = std::chrono::steady_clock::now();
            if (i == 0) {  // the member's start: bytes, no history
                br.seek(map, size, (uint64_t)data0 * 8);
                c.start = (int64_t)data0 * 8;
                take(c.o8.b);
                decode_from(c, br, dec, false);
            } else {
                const auto f0 = std::chrono::steady_clock::now();
                const bool found = find_start(c, dec);
                find_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - f0).count();
                if (found) {
                    br.seek(map, size, c.end);
                    decode_from(c, br, dec, true);
                } else {
                    ++n_nostart;
                }
            }
            const auto d1 = std::chrono::steady_clock::now();
            dec_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d1 - d0).count();
            sym16_n += c.o16.s.n;
            {
                std::lock_guard<std::mutex> g(m);
                c.decoded = true;
            }
            cv.notify_all();
            resolve(i, dec);
            res_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - d1).count();
        }
    }

    // once the previous chunk's window is known: verify this chunk's start (else decode it again
    // from where the previous one ended, with the real history), replace its markers, publish its
    // window, checksum it
    void resolve(size_t i, Decoder& dec) {
        Chunk& c = ch[i];
        const Chunk* pv = nullptr;
        if (i > 0) {
            const auto q0 = std::chrono::steady_clock::now();
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return stop || ch[i - 1].windowed; });
            wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - q0).count();
            if (stop) return;
            pv = &ch[i - 1];
        }
        bool bad = false;
        bool crc_done = false;  // (c.crc holds the resolved bytes' CRC32 already)
        if (pv && (pv->beyond || pv->final_ || pv->error)) {
            c.beyond = true;  // (the stream ended, or failed, before this chunk)
            ++n_beyond;
        } else if (pv && !(c.start >= 0 && (uint64_t)c.start == pv->end)) {
            ++n_redecode;
            // a false start, or none: this chunk decoded again from the previous one's end
            give(c.o16.s);
            c.o16 = Out16();
            give(c.o8.b);
            c.o8 = Out8();
            take(c.o8.b);
            c.o8.b.assign(pv->window.data(), pv->window.size());
            c.o8.win = pv->window.size();
            c.start = (int64_t)pv->end;
            c.end = pv->end;  // (an empty chunk when the previous one's last block ends past this range)
            c.final_ = c.error = false;
            Bits br;
            br.seek(map, size, pv->end);
            decode_from(c, br, dec, false);
        }
        if (!c.beyond) {
            // resolve the markers against the previous window (the stream's bytes before the chunk)
            const std::vector<uint8_t>* w = pv ? &pv->window : nullptr;
            const size_t wn = w ? w->size() : 0;
            const size_t ns = c.o16.s.n;
            take(c.pre);
            c.pre.reserve(ns);
            c.pre.n = ns;
            const uint16_t* src = c.o16.s.p;
            uint8_t* dst = c.pre.p;
            auto one = [&](size_t k) {
                const uint16_t x = src[k];
                if (x < 256) {
                    dst[k] = (uint8_t)x;
                    return true;
                }
                const size_t wi = (size_t)x - 256;  // index into the 32 KiB before the chunk
                if (wi + wn < kWin) return false;   // before the stream's start: zlib's "too far back"
                dst[k] = (*w)[wi + wn - kWin];
                return true;
            };
            const __m128i z = _mm_setzero_si128();
            auto range = [&](size_t k, size_t e) {  // symbols [k, e); false at a marker before the stream
                for (; k + 8 <= e; k += 8) {  // 8 symbols a step; the ones with a marker one by one
                    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + k));
                    if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_srli_epi16(x, 8), z)) == 0xffff) {
                        _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + k), _mm_packus_epi16(x, x));
                        continue;
                    }
                    for (size_t j = k; j < k + 8; ++j)
                        if (!one(j)) {
                            c.pre.n = j;
                            return false;
                        }
                }
                for (; k < e; ++k)
                    if (!one(k)) {
                        c.pre.n = k;
                        return false;
                    }
                return true;
            };
            const size_t n8 = c.o8.b.n - c.o8.win;
            // with a full previous window no marker can point before the stream: only the symbols
            // the window needs are resolved before it is published (the next chunk waits for it),
            // the rest after -- so the chunks' resolutions run side by side, not one after another
            const bool early = wn < kWin;
            size_t t0 = 0;
            std::vector<uint8_t> lut;
            auto fast = [&](size_t k, size_t e) {  // a full window: every symbol is lut[symbol]
                const uint8_t* __restrict t = lut.data();
                // 8 symbols a step: packed as they are when none is a marker (about 2 steps in 3 on
                // FASTQ, where ~18 % of the symbols are markers), else through the table
                for (; k + 8 <= e; k += 8) {
                    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + k));
                    if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_srli_epi16(x, 8), z)) == 0xffff) {
                        _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + k), _mm_packus_epi16(x, x));
                    } else {
                        for (size_t j = k; j < k + 8; ++j) dst[j] = t[src[j]];
                    }
                }
                for (; k < e; ++k) dst[k] = t[src[k]];
            };
            // (a full window: the CRC32 of the resolved bytes is taken slice by slice as they are
            // written, while they are in cache, not in a pass over the chunk afterwards)
            uint32_t crc_tail = 0;
            if (early) {
                bad = !range(0, ns);
            } else {
                lut.resize(256 + kWin);
                for (uint32_t x = 0; x < 256; ++x) lut[x] = (uint8_t)x;
                std::memcpy(lut.data() + 256, w->data(), kWin);
                t0 = ns - std::min(ns, kWin - std::min<size_t>(n8, kWin));
                fast(t0, ns);
                crc_tail = crc_of(dst + t0, ns - t0);
            }
            c.bytes = c.pre.n + n8;
            // window: the last 32 KiB of the stream through this chunk
            std::vector<uint8_t> win;
            const size_t tail8 = std::min<size_t>(n8, kWin);
            const size_t tailp = std::min<size_t>(c.pre.n, kWin - tail8);
            const size_t tailw = std::min<size_t>(wn, kWin - tail8 - tailp);
            win.reserve(tailw + tailp + tail8);
            if (tailw) win.insert(win.end(), w->end() - (ptrdiff_t)tailw, w->end());
            win.insert(win.end(), c.pre.p + c.pre.n - tailp, c.pre.p + c.pre.n);
            win.insert(win.end(), c.o8.b.p + c.o8.b.n - tail8, c.o8.b.p + c.o8.b.n);
            c.window.swap(win);
            if (bad) c.error = true;
            {
                std::lock_guard<std::mutex> g(m);
                c.windowed = true;
            }
            cv.notify_all();
            if (!early) {
                uint32_t x = 0;
                constexpr size_t kSlice = (size_t)64 << 10;
                for (size_t a = 0; a < t0; a += kSlice) {
                    const size_t e = std::min(t0, a + kSlice);
                    fast(a, e);
                    x = crc_more(x, dst + a, e - a);
                }
                c.crc = t0 ? (uint32_t)crc32_combine(x, crc_tail, (z_off_t)(ns - t0)) : crc_tail;
                crc_done = true;
            }
            give(c.o16.s);
        } else {
            {
                std::lock_guard<std::mutex> g(m);
                c.windowed = true;
            }
            cv.notify_all();
        }
        const auto r1 = std::chrono::steady_clock::now();
        if (!c.beyond) {
            uint32_t x = crc_done ? c.crc : crc_of(c.pre.p, c.pre.n);
            const size_t n8 = c.o8.b.n - c.o8.win;
            if (n8) x = (uint32_t)crc32_combine(x, crc_of(c.o8.b.p + c.o8.win, n8), (z_off_t)n8);
            c.crc = x;
        }
        crc_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - r1).count();
        {
            std::lock_guard<std::mutex> g(m);
            c.ready = true;
        }
        cv.notify_all();
    }

    // ---- consumer side ----
    // the next ready chunk's bytes count as good (and, for the final one, the trailer is checked);
    // false when the parallel path gives up here
    bool advance_good(std::unique_lock<std::mutex>& lk, size_t& k) {
        cv.wait(lk, [&] { return ch[k].ready; });
        Chunk& c = ch[k];
        if (c.beyond) return false;  // (cannot happen before the final chunk: checked there)
        if (c.error) return false;
        crc_all = k == 0 ? c.crc : (uint32_t)crc32_combine(crc_all, c.crc, (z_off_t)c.bytes);
        good += c.bytes;
        if (c.final_) {  // the trailer: CRC32, ISIZE, then the end of the file
            const size_t t = (size_t)((c.end + 7) >> 3);
            if (t + 8 != size) return false;
            const uint8_t* q = map + t;
            const uint32_t crc = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
            const uint32_t isz = (uint32_t)q[4] | (uint32_t)q[5] << 8 | (uint32_t)q[6] << 16 | (uint32_t)q[7] << 24;
            if (crc != crc_all || isz != (uint32_t)good) return false;
            finished = true;
        } else if (k + 1 >= ch.size()) {
            return false;  // the data ends without a final block
        }
        return true;
    }

    void start_fallback() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
            anomaly = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
        th.clear();
        fb = true;
        gz = gzopen(path.c_str(), "r");
        if (!gz) {
            fb_bad = fb_end = true;
            return;
        }
        // (zlib's default buffer, as the reference's FqReader: each gzread inflates into the caller's
        // buffer, so an error fails the call whose bytes it lies in)
        // skip what went out already (the same bytes: a prefix of the stream gzread gives)
        std::vector<char> tmp(call);
        uint64_t skip = handed;
        while (skip > 0) {
            const int r = gzread(gz, tmp.data(), (unsigned)call);
            if (r < 0) {
                fb_bad = fb_end = true;
                return;
            }
            const uint64_t take = std::min<uint64_t>(skip, (uint64_t)r);
            skip -= take;
            if ((size_t)r > take) fb_buf.assign(tmp.data() + take, tmp.data() + r);
            if ((size_t)r < call) {
                fb_end = true;
                return;
            }
        }
    }

    bool fb_read(char* dst, size_t want, size_t& got) {
        got = 0;
        while (got < want) {
            if (fb_off < fb_buf.size()) {
                const size_t n = std::min(want - got, fb_buf.size() - fb_off);
                std::memcpy(dst + got, fb_buf.data() + fb_off, n);
                fb_off += n;
                got += n;
                continue;
            }
            if (fb_end) break;
            fb_buf.resize(call);
            fb_off = 0;
            const int r = gzread(gz, fb_buf.data(), (unsigned)call);
            if (r < 0) {
                fb_buf.clear();
                fb_bad = fb_end = true;
                break;
            }
            fb_buf.resize((size_t)r);
            if ((size_t)r < call) fb_end = true;
        }
        if (fb_bad && fb_off >= fb_buf.size() && !reported) {
            reported = true;
            return false;
        }
        return true;
    }

    int nthreads = 1;
    bool started = false;
    void start() {  // (the workers start at the first read: a source opened and never read costs nothing)
        started = true;
        for (int t = 0; t < nthreads; ++t) th.emplace_back([this] { work(); });
    }

    bool read(char* dst, size_t want, size_t& got) {
        if (!started) start();
        if (fb) return fb_read(dst, want, got);
        got = 0;
        std::unique_lock<std::mutex> lk(m);
        while (got < want) {
            if (cur >= ch.size()) break;
            // bytes may go out up to the last call boundary before what is verified, or all of
            // them once the member's trailer checked out
            // (good - 1: zlib parses the next block's header, or the trailer, within the call that
            // ends exactly at a block end, so an error there fails that call)
            const uint64_t limit = finished ? good : good ? (good - 1) / call * call : 0;
            if (handed >= limit) {
                if (finished) break;
                size_t k = next_good;
                if (k >= ch.size() || !advance_good(lk, k)) {
                    lk.unlock();
                    start_fallback();
                    size_t g2 = 0;
                    const bool ok = fb_read(dst + got, want - got, g2);
                    got += g2;
                    return ok;
                }
                next_good = k + 1;
                cv.notify_all();
                continue;
            }
            Chunk& c = ch[cur];
            const size_t n8 = c.o8.b.n - c.o8.win;
            if (cur_pos >= c.bytes) {  // done with it: free it, let a worker take another
                give(c.pre);
                give(c.o8.b);
                ++cur;
                cur_pos = 0;
                consumed = cur;
                cv.notify_all();
                continue;
            }
            size_t n = (size_t)std::min<uint64_t>(want - got, limit - handed);
            if (cur_pos < c.pre.n) {
                n = std::min(n, c.pre.n - cur_pos);
                std::memcpy(dst + got, c.pre.p + cur_pos, n);
            } else {
                const size_t o = cur_pos - c.pre.n;
                n = std::min(n, n8 - o);
                std::memcpy(dst + got, c.o8.b.p + c.o8.win + o, n);
            }
            cur_pos += n;
            got += n;
            handed += n;
        }
        return true;
    }
    size_t next_good = 0;
};

template <>
std::vector<PodBuf<uint8_t>>& ParGzSource::Impl::pool_of<uint8_t>() {
    return pool8;
}
template <>
std::vector<PodBuf<uint16_t>>& ParGzSource::Impl::pool_of<uint16_t>() {
    return pool16;
}

std::unique_ptr<ParGzSource> ParGzSource::open(const std::string& path, size_t call, int threads) {
    return open_chunked(path, call, threads, 0);
}

std::unique_ptr<ParGzSource> ParGzSource::open_chunked(const std::string& path, size_t call, int threads, size_t chunk) {
    const char* env = std::getenv("FQ_PARGZ");
    if (env && std::string(env) == "0") return nullptr;
    const char* ce = std::getenv("FQ_PARGZ_CHUNK");  // (tests: small chunks)
    if (!chunk) chunk = ce && std::atoll(ce) > 0 ? (size_t)std::atoll(ce) : (size_t)4 << 20;
    chunk = std::max<size_t>(chunk, 4096);
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || (size_t)st.st_size < 2 * chunk) {
        ::close(fd);
        return nullptr;
    }
    void* mp = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (mp == MAP_FAILED) return nullptr;
    madvise(mp, (size_t)st.st_size, MADV_SEQUENTIAL);
    std::unique_ptr<Impl> im(new Impl);
    im->map = static_cast<const uint8_t*>(mp);
    im->size = (size_t)st.st_size;
    im->data0 = member_data(im->map, im->size, 0);
    if (!im->data0) return nullptr;  // (Impl unmaps)
    im->call = std::max<size_t>(call, 1);
    im->path = path;
    const size_t body = im->size - im->data0;
    const size_t nch = std::max<size_t>(1, body / chunk);
    im->ch.resize(nch);
    for (size_t i = 0; i < nch; ++i) {
        im->ch[i].nom0 = (uint64_t)(im->data0 + body * i / nch) * 8;
        im->ch[i].nom1 = i + 1 < nch ? (uint64_t)(im->data0 + body * (i + 1) / nch) * 8 : (uint64_t)im->size * 8;
    }
    const int nt = std::max(1, threads);
    const char* ae = std::getenv("FQ_PARGZ_AHEAD");  // (profiling: chunks ahead per thread)
    im->ahead = (size_t)std::max(4, (ae && std::atoi(ae) > 0 ? std::atoi(ae) : 2) * nt);
    Impl* p = im.get();
    p->nthreads = nt;
    return std::unique_ptr<ParGzSource>(new ParGzSource(im.release()));
}

bool ParGzSource::read(char* dst, size_t want, size_t& got) { return p_->read(dst, want, got); }

bool ParGzSource::fell_back() const { return p_->fb; }

void ParGzSource::prefetch() {
    if (!p_->started) p_->start();
}

ParGzSource::~ParGzSource() { delete p_; }

bool pargz_read_all(const std::string& path, size_t call, int threads, size_t chunk, std::string& out, bool& ok,
                    std::string& how) {
    std::unique_ptr<ParGzSource> s = ParGzSource::open_chunked(path, call, threads, chunk);
    if (!s) return false;
    out.clear();
    ok = true;
    std::vector<char> buf(call);
    for (;;) {
        size_t got = 0;
        const bool r = s->read(buf.data(), buf.size(), got);
        out.append(buf.data(), got);
        if (!r) {
            ok = false;
            break;
        }
        if (got == 0) break;
    }
    how = s->fell_back() ? "zlib fallback" : "parallel";
    return true;
}

}  // namespace fqhost

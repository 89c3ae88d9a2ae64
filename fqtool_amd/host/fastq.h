// fastq.h -- FASTQ input and output of the host tool.
//
// FqReader restates the reference reader (src/fqreader.cpp:3-195): 1 MiB buffered lines over
// zlib or stdio, a line ends at '\r' or '\n' ("\r\n" counts once, except at a buffer's last
// byte), records start at the next line beginning with '@', phred64 qualities are shifted at
// parse time (src/read.h:71-75) and a quality/sequence length mismatch ends the input
// (src/fqreader.cpp:184-191).  Unlike the reference it builds no std::string per field: records
// are appended to a pack's text arena and addressed by offsets.
//
// A Pack holds the records' text (per mate: name, seq, strand, qual back to back) and the
// engine's batch planes (chunk-interleaved tiles, include/fqengine.h), which pack_tiles fills
// from the text on a thread pool.  Writer restates src/writer.cpp (gzip level -z or plain).
#pragma once

#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fqengine.h"

namespace fqhost {

// Growable byte buffer that keeps its capacity when cleared (packs are recycled) and does not
// zero what it allocates.  A pinned buffer takes page-locked memory from the engine
// (fq_host_alloc: the H2D/D2H DMA then overlaps the kernels); without a HIP device it silently
// uses ordinary memory, which the engine also accepts (synchronous copies).
class ByteBuf {
   public:
    explicit ByteBuf(bool pinned = false) : want_pinned_(pinned) {}
    ~ByteBuf() { release(); }
    ByteBuf(const ByteBuf&) = delete;
    ByteBuf& operator=(const ByteBuf&) = delete;
    ByteBuf(ByteBuf&& o) noexcept { *this = std::move(o); }
    ByteBuf& operator=(ByteBuf&& o) noexcept;
    char* data() { return p_; }
    const char* data() const { return p_; }
    size_t size() const { return size_; }
    void clear() { size_ = 0; }
    void resize_uninit(size_t n) {
        reserve(n);
        size_ = n;
    }
    void reserve(size_t n);
    char* extend(size_t n) {  // appends n uninitialised bytes, returns their start
        if (size_ + n > cap_) reserve(std::max(size_ + n, cap_ + cap_ / 2 + 4096));
        char* r = p_ + size_;
        size_ += n;
        return r;
    }
    void truncate(size_t n) { size_ = n; }
    bool pinned() const { return is_pinned_; }

   private:
    void release();
    char* p_ = nullptr;
    size_t size_ = 0, cap_ = 0;
    bool want_pinned_ = false, is_pinned_ = false;
};

// Array of T over a ByteBuf (read lengths, result records): pinned like its buffer.
template <class T>
class PodBuf {
   public:
    explicit PodBuf(bool pinned = false) : b_(pinned) {}
    void resize(size_t n) { b_.resize_uninit(n * sizeof(T)); }
    void clear() { b_.clear(); }
    size_t size() const { return b_.size() / sizeof(T); }
    T* data() { return reinterpret_cast<T*>(b_.data()); }
    const T* data() const { return reinterpret_cast<const T*>(b_.data()); }
    T& operator[](size_t i) { return data()[i]; }
    const T& operator[](size_t i) const { return data()[i]; }
    const T* begin() const { return data(); }
    const T* end() const { return data() + size(); }

   private:
    ByteBuf b_;
};

// One record's fields in a mate's text arena: name at off, then seq (len bytes), strand, qual.
struct Rec {
    uint64_t off;
    uint32_t name_len, strand_len, len;
};

class FqReader {
   public:
    FqReader(const std::string& path, bool phred64);
    ~FqReader();
    FqReader(const FqReader&) = delete;
    FqReader& operator=(const FqReader&) = delete;
    // Next record appended to `text`; false at end of input or on a quality/sequence length
    // mismatch, whose message (the reference's, src/fqreader.cpp:185-190) is left in error().
    bool read(ByteBuf& text, Rec& r);
    // Same, as strings (the evaluator pre-pass); prints a mismatch message like the reference.
    bool read(std::string& name, std::string& seq, std::string& strand, std::string& qual);
    const std::string& error() const { return err_; }

   private:
    void get_line(ByteBuf& out);
    void fill();
    bool at_eof() const { return eof_; }
    gzFile gz_ = nullptr;
    FILE* fp_ = nullptr;
    bool phred64_;
    std::vector<char> buf_;
    int len_ = 0, used_ = 0;
    bool eof_ = false;
    std::string err_;
    ByteBuf scratch_;  // the string overload's record
};

// Minimal fork-join pool: run(n, fn) calls fn(0..n-1) on the workers and the calling thread and
// returns when all are done.  Several threads may call run concurrently.
class Pool {
   public:
    explicit Pool(int workers);
    ~Pool();
    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;
    void run(int n, const std::function<void(int)>& fn);
    int size() const { return workers_ + 1; }

   private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
    int workers_;
};

// One pack of reads (pairs when paired): record text + the engine's batch planes + the engine's
// per-read records.  A pinned pack keeps planes, lengths and records in page-locked memory.
struct Pack {
    explicit Pack(bool pinned = false)
        : seq{ByteBuf(pinned), ByteBuf(pinned)},
          qual{ByteBuf(pinned), ByteBuf(pinned)},
          len{PodBuf<uint16_t>(pinned), PodBuf<uint16_t>(pinned)},
          res(pinned) {}
    int n = 0;
    int stride = 0;
    bool paired = false;
    ByteBuf text[2];
    std::vector<Rec> rec[2];
    ByteBuf seq[2], qual[2];  // batch planes
    PodBuf<uint16_t> len[2];
    PodBuf<fq_read_result> res;  // engine records: n (SE) or 2n (PE)
    uint64_t seq_no = 0;

    const char* name(int m, size_t i) const { return text[m].data() + rec[m][i].off; }
    const char* seq_text(int m, size_t i) const { return name(m, i) + rec[m][i].name_len; }
    const char* strand(int m, size_t i) const { return seq_text(m, i) + rec[m][i].len; }
    const char* qual_text(int m, size_t i) const { return strand(m, i) + rec[m][i].strand_len; }
    void clear();
    fq_batch batch() const;
    fq_read_result* results() {  // sized for this pack
        res.resize((size_t)n * (paired ? 2 : 1));
        return res.data();
    }
};

// Fills the pack's lengths, stride and tile planes from its record text (pool-parallel over
// whole tiles when a pool is given).  Throws on reads longer than 65535 bases.
void pack_tiles(Pack& pk, Pool* pool);

// Reads up to max_n records (pairs) into a pack and builds its planes.  Two-file PE input is
// parsed by two threads, one per mate, with the reference's stop rule and messages (the pair
// reader stops at the first mate that fails, src/fqreader.cpp:254-267).
// Returns false when no record could be read.
class PackReader {
   public:
    PackReader(const std::string& in1, const std::string& in2, bool interleaved, bool phred64);
    bool next(Pack& pk, size_t max_n, Pool* pool = nullptr);
    bool paired() const { return paired_; }
    uint64_t reads_seen() const { return reads_; }

   private:
    FqReader r1_;
    FqReader* r2_ = nullptr;
    std::unique_ptr<FqReader> r2_own_;
    bool paired_, interleaved_;
    bool done_ = false;
    uint64_t reads_ = 0, packs_ = 0;
};

// An output file.  Plain files take the text as is.  Gzip output (src/writer.cpp:36-47, level
// -z) is one gzip member per block of text, the blocks compressed independently (in parallel
// on a pool when one is given): a valid multi-member gzip file whose decompressed bytes are the
// reference's.
class Writer {
   public:
    Writer(const std::string& path, int level);
    ~Writer();
    Writer(const Writer&) = delete;
    Writer& operator=(const Writer&) = delete;
    void write(const std::vector<std::string>& blocks, Pool* pool = nullptr);
    void write(const std::string& s) { write(std::vector<std::string>{s}); }
    void close();  // flushes; throws on a short write or a failed close (full disk)

   private:
    FILE* fp_ = nullptr;
    bool gzip_ = false;
    bool any_member_ = false;
    int level_ = 4;
};

}  // namespace fqhost

// pargz.h -- single-stream gzip input inflated on several threads.
//
// The reference reads every .gz input through zlib's gzread in 1 MiB calls (src/fqreader.cpp:3-47),
// one thread per file.  A plain gzip file is one deflate stream, so its blocks cannot be located
// from the headers (as BGZF members can, BgzfSource): here the compressed file is cut into chunks,
// each worker finds the first deflate block that starts in its chunk by trying bit offsets (a
// dynamic-Huffman block header that builds valid codes and whose block decodes), and decodes from
// there with 16-bit symbols in which a reference into the unknown 32 KiB before the chunk is a
// marker.  Once the previous chunk is known the chunk's start is verified (the previous chunk's
// decode must have ended exactly there -- otherwise the chunk is decoded again from where it ended,
// with the real window) and its markers are replaced by the window's bytes.  The published
// speculative two-pass method of pugz (Kerbiriou & Chikhi 2019) and rapidgzip (Knespel & Brunst
// 2023), restated here; no code from either.
//
// The byte stream handed out is the one gzread gives.  Bytes go out only up to the last gzread
// call boundary before the end of what is decoded and verified; anything the parallel path does not
// take as a clean single member -- a data error, a CRC32 / ISIZE mismatch, data after the member,
// a member that ends early -- hands the file to zlib's stream reader from its start, which skips
// the bytes already handed out: the reference's truncation semantics on corrupt input stay exact.
#pragma once

#include <cstddef>
#include <memory>
#include <string>

namespace fqhost {

class ParGzSource {
   public:
    // nullptr unless `path` is a regular gzip file large enough to split (FQ_PARGZ=0: never);
    // `call`: the reference's gzread size; `threads`: decoding threads for this file
    static std::unique_ptr<ParGzSource> open(const std::string& path, size_t call, int threads);
    // the same with chunks of `chunk` compressed bytes (0: the default, FQ_PARGZ_CHUNK or 4 MiB)
    static std::unique_ptr<ParGzSource> open_chunked(const std::string& path, size_t call, int threads, size_t chunk);
    // up to `want` more bytes of the decompressed stream into dst; false on corrupt data, once the
    // bytes the reference's gzread calls would have returned before the failing one are handed out
    bool read(char* dst, size_t want, size_t& got);
    // start the decoding threads now (otherwise they start at the first read)
    void prefetch();
    ~ParGzSource();
    bool fell_back() const;  // the stream went to zlib's reader (an anomaly, or several members)
    struct Impl;

   private:
    explicit ParGzSource(Impl* i) : p_(i) {}
    Impl* p_;
};

// Test entry (fqh_pargz_read_all, capi.cpp): the whole stream of `path` through ParGzSource with the
// given chunk size (compressed bytes), as read() hands it out; *ok = 0 when read() reported corrupt
// data.  Returns false when the parallel path does not apply (the caller then compares nothing).
bool pargz_read_all(const std::string& path, size_t call, int threads, size_t chunk, std::string& out, bool& ok,
                    std::string& how);

}  // namespace fqhost

// fastq.cpp -- see fastq.h.
#include "fastq.h"

#include <algorithm>
#include <cstring>
#include <iostream>
#include <memory>
#include <stdexcept>

namespace fqhost {

namespace {
constexpr int kBufSize = 1 << 20;  // src/fqreader.cpp:10

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}
}  // namespace

FqReader::FqReader(const std::string& path, bool phred64) : phred64_(phred64), buf_(kBufSize) {
    if (ends_with(path, ".gz")) {
        gz_ = gzopen(path.c_str(), "r");
        if (!gz_) throw std::runtime_error("Failed to open file: " + path);
        gzrewind(gz_);
    } else {
        fp_ = path == "/dev/stdin" ? stdin : std::fopen(path.c_str(), "rb");
        if (!fp_) throw std::runtime_error("Failed to open file: " + path);
    }
    fill();
}

FqReader::~FqReader() {
    if (gz_) gzclose(gz_);
    if (fp_ && fp_ != stdin) std::fclose(fp_);
}

void FqReader::fill() {  // FqReader::readToBuf, src/fqreader.cpp:30-44
    if (gz_) {
        len_ = gzread(gz_, buf_.data(), kBufSize);
        if (len_ < 0) {
            std::cerr << "Error to read gzip file" << std::endl;
            len_ = 0;
        }
        eof_ = gzeof(gz_) != 0 || len_ < kBufSize;
    } else {
        len_ = (int)std::fread(buf_.data(), 1, kBufSize, fp_);
        eof_ = std::feof(fp_) != 0 || len_ < kBufSize;
    }
    used_ = 0;
}

bool FqReader::at_eof() const { return eof_; }

// FqReader::getLine, src/fqreader.cpp:90-150
bool FqReader::get_line(std::string& out) {
    int start = used_, end = start;
    while (end < len_ && buf_[end] != '\r' && buf_[end] != '\n') ++end;
    if (end < len_ || len_ < kBufSize) {
        out.assign(buf_.data() + std::min(start, len_), (size_t)std::max(0, end - start));
        ++end;
        if (end < len_ - 1 && buf_[end] == '\n') ++end;
        used_ = end;
        return true;
    }
    out.assign(buf_.data() + start, (size_t)(len_ - start));
    for (;;) {
        fill();
        start = 0;
        end = 0;
        while (end < len_ && buf_[end] != '\r' && buf_[end] != '\n') ++end;
        if (end < len_ || len_ < kBufSize) {
            out.append(buf_.data() + start, (size_t)(end - start));
            ++end;
            if (end < len_ - 1 && buf_[end] == '\n') ++end;
            used_ = end;
            return true;
        }
        out.append(buf_.data() + start, (size_t)(len_ - start));
    }
}

// FqReader::read, src/fqreader.cpp:160-195
bool FqReader::read(std::string& name, std::string& seq, std::string& strand, std::string& qual) {
    if (used_ >= len_ && at_eof()) return false;
    get_line(name);
    while ((name.empty() && !(used_ >= len_ && at_eof())) || (!name.empty() && name[0] != '@')) get_line(name);
    if (name.empty()) return false;
    get_line(seq);
    get_line(strand);
    get_line(qual);
    if (qual.size() != seq.size()) {
        std::cerr << "Error: base sequnce and quality sequence have different length: \n"
                  << name << "\n" << seq << "\n" << qual << "\n" << strand << "\n";
        return false;
    }
    if (phred64_)  // Read::convertPhread64To33, src/read.h:71-75 (char arithmetic)
        for (char& c : qual) c = (char)std::max(33, (int)c - (64 - 33));
    return true;
}

fq_batch Pack::batch() const {
    fq_batch b;
    b.n = n;
    b.stride = stride;
    b.seq1 = seq[0].data();
    b.qual1 = qual[0].data();
    b.len1 = len[0].data();
    b.seq2 = paired ? seq[1].data() : nullptr;
    b.qual2 = paired ? qual[1].data() : nullptr;
    b.len2 = paired ? len[1].data() : nullptr;
    return b;
}

PackReader::PackReader(const std::string& in1, const std::string& in2, bool interleaved, bool phred64)
    : r1_(in1, phred64), paired_(!in2.empty() || interleaved), interleaved_(interleaved) {
    if (!in2.empty() && !interleaved) {
        r2_own_.reset(new FqReader(in2, phred64));
        r2_ = r2_own_.get();
    } else if (interleaved) {
        r2_ = &r1_;
    }
}

bool PackReader::next(Pack& pk, size_t max_n) {
    if (done_) return false;
    const int mates = paired_ ? 2 : 1;
    pk.paired = paired_;
    pk.n = 0;
    for (int m = 0; m < 2; ++m) {
        pk.name[m].clear();
        pk.strand[m].clear();
        pk.seq_text[m].clear();
        pk.qual_text[m].clear();
    }
    size_t maxlen = 0;
    std::string nm, sq, sd, ql;
    while ((size_t)pk.n < max_n) {
        bool ok = true;
        std::string names[2], seqv[2], strands[2], qualv[2];
        for (int m = 0; m < mates && ok; ++m) {  // FqReaderPair::read, src/fqreader.cpp:254-267
            FqReader* r = m == 0 ? &r1_ : r2_;
            ok = r->read(names[m], seqv[m], strands[m], qualv[m]);
        }
        if (!ok) {
            done_ = true;
            break;
        }
        for (int m = 0; m < mates; ++m) {
            maxlen = std::max(maxlen, seqv[m].size());
            pk.name[m].push_back(std::move(names[m]));
            pk.strand[m].push_back(std::move(strands[m]));
            pk.seq_text[m].push_back(std::move(seqv[m]));
            pk.qual_text[m].push_back(std::move(qualv[m]));
        }
        ++pk.n;
    }
    if (pk.n == 0) return false;
    if (maxlen > 65535) throw std::runtime_error("read longer than 65535 bases");
    pk.stride = (int)std::max<size_t>(16, (maxlen + 15) & ~(size_t)15);
    for (int m = 0; m < mates; ++m) {
        const size_t bytes = fq_batch_bytes(pk.n, pk.stride);
        pk.seq[m].assign(bytes, 0);
        pk.qual[m].assign(bytes, 0);
        pk.len[m].resize((size_t)pk.n);
        for (int i = 0; i < pk.n; ++i) {
            const std::string& s = pk.seq_text[m][i];
            const std::string& q = pk.qual_text[m][i];
            // chunk-interleaved tiles: 16-byte pieces of the row, 512 bytes apart
            for (size_t j = 0; j < s.size(); j += FQ_CHUNK) {
                const size_t k = std::min<size_t>(FQ_CHUNK, s.size() - j);
                const size_t o = fq_batch_offset(pk.stride, i, (int32_t)j);
                std::memcpy(&pk.seq[m][o], s.data() + j, k);
                std::memcpy(&pk.qual[m][o], q.data() + j, k);
            }
            pk.len[m][i] = (uint16_t)s.size();
        }
    }
    if (!paired_) {
        pk.seq[1].clear();
        pk.qual[1].clear();
        pk.len[1].clear();
    }
    pk.seq_no = packs_++;
    reads_ += (uint64_t)pk.n * mates;
    return true;
}

Writer::Writer(const std::string& path, int level) {
    if (ends_with(path, ".gz")) {  // src/writer.cpp:36-47
        gz_ = gzopen(path.c_str(), "w");
        if (!gz_) throw std::runtime_error("cannot open " + path);
        gzsetparams(gz_, level, Z_DEFAULT_STRATEGY);
        gzbuffer(gz_, 1024 * 1024);
    } else {
        fp_ = std::fopen(path.c_str(), "wb");
        if (!fp_) throw std::runtime_error("cannot open " + path);
    }
}

Writer::~Writer() {
    if (gz_) gzclose(gz_);
    if (fp_) std::fclose(fp_);
}

void Writer::write(const std::string& s) {
    if (s.empty()) return;
    if (gz_) gzwrite(gz_, s.data(), (unsigned)s.size());
    else std::fwrite(s.data(), 1, s.size(), fp_);
}

}  // namespace fqhost

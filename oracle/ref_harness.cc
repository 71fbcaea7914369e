// ref_harness.cc -- TEST INFRASTRUCTURE ONLY.
//
// Thin extern "C" wrapper around the reference's OWN Snappy sources, which
// oracle/Makefile compiles in place from /root/reference/flare/io/snappy/
// (nothing is copied into this repo).  The output, oracle/_ref/
// libsnappy_ref.so, is git-ignored; it validates the C restatement
// (snappy_oracle.c), generates tests/golden/, and is the "reference" CPU
// baseline timed by bench.py.
//
// The Source/Sink classes below reproduce what flare's cord_buf adapters
// hand to the codec (flare/io/cord_buf.h:624-665, cord_buf.cc:2018-2071):
//   * the source yields fixed-size fragments (cord_buf blocks carry 8160
//     payload bytes, cord_buf.h:67) and Peek never repositions;
//   * the sink copies on Append, offers a block only for <= 8000-byte
//     GetAppendBuffer requests, and does NOT override
//     GetAppendBufferVariable, so decode takes the SnappyScatteredWriter path
//     (snappy.cc:1558-1561) exactly as policy::SnappyDecompress does.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "flare/io/snappy/snappy-sinksource.h"
#include "flare/io/snappy/snappy.h"

namespace {

class FragmentSource : public flare::snappy::Source {
 public:
  FragmentSource(const char* p, size_t n, size_t frag)
      : p_(p), left_(n), frag_(frag ? frag : n), in_frag_(0) {}
  size_t Available() const override { return left_; }
  const char* Peek(size_t* len) override {
    // Bytes remaining in the current fragment, like a cord_buf BlockRef.
    size_t room = frag_ - in_frag_;
    *len = std::min(room, left_);
    return p_;
  }
  void Skip(size_t n) override {
    while (n > 0) {
      size_t room = frag_ - in_frag_;
      size_t k = std::min(room, n);
      p_ += k;
      left_ -= k;
      n -= k;
      in_frag_ += k;
      if (in_frag_ == frag_) in_frag_ = 0;
    }
  }

 private:
  const char* p_;
  size_t left_;
  size_t frag_;
  size_t in_frag_;
};

// Copying sink into a caller buffer with a capacity guard.
class CopySink : public flare::snappy::Sink {
 public:
  CopySink(char* dst, size_t cap) : dst_(dst), cap_(cap), n_(0) {}
  void Append(const char* bytes, size_t n) override {
    size_t k = n_ + n <= cap_ ? n : (n_ < cap_ ? cap_ - n_ : 0);
    if (k) memcpy(dst_ + n_, bytes, k);
    n_ += n;
  }
  char* GetAppendBuffer(size_t length, char* scratch) override {
    return length <= 8000 ? block_ : scratch;
  }
  size_t size() const { return n_; }

 private:
  char* dst_;
  size_t cap_;
  size_t n_;
  char block_[8000];
};

}  // namespace

extern "C" {

size_t ref_max_compressed_length(size_t n) {
  return flare::snappy::MaxCompressedLength(n);
}

// snappy::Compress(Source*, Sink*) via fragmenting source (frag = Peek size).
size_t ref_compress(const char* in, size_t n, char* out, size_t frag) {
  FragmentSource src(in, n, frag);
  CopySink sink(out, flare::snappy::MaxCompressedLength(n));
  return flare::snappy::Compress(&src, &sink);
}

// snappy::Uncompress(Source*, Sink*).  Returns 1/0 (reference bool);
// *produced = bytes the sink received (partial output on failure).
int ref_uncompress(const char* in, size_t n, char* out, size_t cap,
                   size_t* produced, size_t frag) {
  FragmentSource src(in, n, frag);
  CopySink sink(out, cap);
  bool ok = flare::snappy::Uncompress(&src, &sink);
  *produced = sink.size();
  return ok ? 1 : 0;
}

// Flat API: GetUncompressedLength (strict) + RawUncompress.
int ref_get_uncompressed_length(const char* in, size_t n, size_t* ulen) {
  return flare::snappy::GetUncompressedLength(in, n, ulen) ? 1 : 0;
}
int ref_raw_uncompress(const char* in, size_t n, char* out) {
  return flare::snappy::RawUncompress(in, n, out) ? 1 : 0;
}
// snappy::UncompressAsMuchAsPossible(Source*, Sink*) (snappy.cc:1530-1535):
// returns its result; *got = the bytes the sink received.
size_t ref_uncompress_as_much(const char* in, size_t n, char* out, size_t cap, size_t frag,
                              size_t* got) {
  FragmentSource src(in, n, frag);
  CopySink sink(out, cap);
  const size_t r = flare::snappy::UncompressAsMuchAsPossible(&src, &sink);
  *got = sink.size();
  return r;
}
// snappy::RawUncompressToIOVec(const char*, size_t, const iovec*, size_t)
// (snappy.cc:1122-1132): the reference's bool; the iovecs as it leaves them.
int ref_uncompress_iovec(const char* in, size_t n, char* const* base, const size_t* len,
                         size_t cnt) {
  std::vector<flare::snappy::iovec> iov(cnt ? cnt : 1);
  for (size_t i = 0; i < cnt; ++i) {
    iov[i].iov_base = base[i];
    iov[i].iov_len = len[i];
  }
  return flare::snappy::RawUncompressToIOVec(in, n, iov.data(), cnt) ? 1 : 0;
}
int ref_is_valid(const char* in, size_t n) {
  return flare::snappy::IsValidCompressedBuffer(in, n) ? 1 : 0;
}
int ref_get_uncompressed_length_source(const char* in, size_t n,
                                       uint32_t* ulen) {
  FragmentSource src(in, n, 0);
  return flare::snappy::GetUncompressedLength(&src, ulen) ? 1 : 0;
}

// CPU baseline: the handler's per-message path (fragmenting source, copying
// sink, scattered decode) over a batch, threads owning strided indices.
// mode 0 = compress, 1 = decompress.  Returns wall seconds.
double ref_batch(int mode, const char* in, const uint64_t* in_off,
                 const uint32_t* in_len, uint32_t n_msgs, char* out,
                 const uint64_t* out_off, const uint32_t* out_cap,
                 uint32_t* out_len, int n_threads, size_t frag) {
  if (n_threads < 1) n_threads = 1;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) {
    th.emplace_back([=]() {
      for (uint32_t i = t; i < n_msgs; i += n_threads) {
        FragmentSource src(in + in_off[i], in_len[i], frag);
        if (mode == 0) {
          CopySink sink(out + out_off[i],
                        flare::snappy::MaxCompressedLength(in_len[i]));
          out_len[i] = (uint32_t)flare::snappy::Compress(&src, &sink);
        } else {
          CopySink sink(out + out_off[i], out_cap[i]);
          bool ok = flare::snappy::Uncompress(&src, &sink);
          out_len[i] = ok ? (uint32_t)sink.size() : 0xffffffffu;
        }
      }
    });
  }
  for (auto& x : th) x.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
      .count();
}

}  // extern "C"

// test_rpc_snappy_compress.cc -- the reference's snappy handler tests
// (/root/reference/test/rpc/rpc_snappy_compress_test.cc) re-run against the
// GPU-backed handler, plus registry / cord_buf / batching cases.
//   ./test_rpc_snappy_compress --cpu   tests that need no GPU
//   ./test_rpc_snappy_compress --gpu   codec tests (MI355X)
#include <hip/hip_runtime.h>
#include <sys/uio.h>

#include <condition_variable>
#include <mutex>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "compress.h"
#include "cord_buf.h"
#include "gpu_codec.h"
#include "lz4_compress.h"
#include "snappy.h"
#include "snappy_compress.h"
#include "snappy_message.h"

namespace {
struct TestCase {
  const char* name;
  bool gpu;
  std::function<void()> fn;
};
std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Reg {
  Reg(const char* n, bool g, std::function<void()> f) { registry().push_back({n, g, std::move(f)}); }
};
int g_failures = 0;
struct Failure {};
}  // namespace

#define TEST_CPU(name) static void name(); static Reg reg_##name(#name, false, name); static void name()
#define TEST_GPU(name) static void name(); static Reg reg_##name(#name, true, name); static void name()
#define ASSERT_TRUE(c)                                                         \
  do {                                                                         \
    if (!(c)) {                                                                \
      fprintf(stderr, "  %s:%d: ASSERT_TRUE(%s) failed\n", __FILE__, __LINE__, #c); \
      throw Failure{};                                                         \
    }                                                                          \
  } while (0)
#define ASSERT_FALSE(c) ASSERT_TRUE(!(c))
#define ASSERT_EQ(a, b) ASSERT_TRUE((a) == (b))

using flare::cord_buf;
using namespace flare::rpc;

static std::string pattern(int len, bool digits) {  // the reference tests' text loops
  std::string t;
  while ((int)t.size() < len) {
    for (int i = 0; i < 26 && (int)t.size() < len; i++) t.push_back('a' + i);
    if (digits)
      for (int i = 0; i < 10 && (int)t.size() < len; i++) t.push_back('0' + i);
  }
  return t;
}

static std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : s) { o.push_back(d[c >> 4]); o.push_back(d[c & 15]); }
  return o;
}

// ------------------------------------------------------------------ CPU tests
TEST_CPU(registry_semantics) {
  ResetCompressHandlersForTesting();
  ASSERT_EQ(std::string(CompressTypeToCStr(COMPRESS_TYPE_NONE)), "none");
  ASSERT_EQ(std::string(CompressTypeToCStr(COMPRESS_TYPE_SNAPPY)), "unknown");
  ASSERT_EQ(RegisterCompressHandler(COMPRESS_TYPE_SNAPPY, CompressHandler{nullptr, nullptr, "x"}), -1);
  ASSERT_EQ(RegisterCompressHandler((CompressType)1024,
                                    CompressHandler{policy::SnappyCompress, policy::SnappyDecompress, "x"}),
            -1);
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  ASSERT_EQ(std::string(CompressTypeToCStr(COMPRESS_TYPE_SNAPPY)), "snappy");
  // second registration of the same type is rejected (FATAL in the reference)
  ASSERT_EQ(RegisterCompressHandler(COMPRESS_TYPE_SNAPPY,
                                    CompressHandler{policy::SnappyCompress, policy::SnappyDecompress, "s"}),
            -1);
  std::vector<CompressHandler> v;
  ListCompressHandler(&v);
  ASSERT_EQ(v.size(), 1u);
  ASSERT_TRUE(FindCompressHandler(COMPRESS_TYPE_LZ4) == nullptr);  // LZ4: no handler
  snappy_message::SnappyMessageProto m;
  cord_buf b;
  ASSERT_FALSE(SerializeAsCompressedData(m, &b, COMPRESS_TYPE_GZIP));  // not registered
  m.set_text("plain");
  ASSERT_TRUE(SerializeAsCompressedData(m, &b, COMPRESS_TYPE_NONE));
  snappy_message::SnappyMessageProto m2;
  ASSERT_TRUE(ParseFromCompressedData(b, &m2, COMPRESS_TYPE_NONE));
  ASSERT_EQ(m2.text(), "plain");
}

// COMPRESS_TYPE_LZ4 (options.proto:74): no reference handler; ours on the
// host codec.  Known answer: varint(200) + liblz4 1.9.3's block of the
// reference tests' 200-byte text loop.
TEST_CPU(lz4_handler) {
  ASSERT_EQ(GlobalInitializeLz4(), 0);
  ASSERT_EQ(std::string(CompressTypeToCStr(COMPRESS_TYPE_LZ4)), "lz4");
  ASSERT_TRUE(FindCompressHandler(COMPRESS_TYPE_LZ4) != nullptr);
  cord_buf in, out, back;
  in.append(pattern(200, true));
  ASSERT_TRUE(policy::Lz4Compress(in, &out));
  ASSERT_EQ(hex(out.to_string()),
            "c801ff156162636465666768696a6b6c6d6e6f707172737475767778797a3031323334353637383924008c507071727374");
  ASSERT_TRUE(policy::Lz4Decompress(out, &back));
  ASSERT_EQ(back.to_string(), pattern(200, true));
  snappy_message::SnappyMessageProto m, m2;
  m.set_text(pattern(12435, true));
  for (int i = 0; i < 3; ++i) m.add_numbers(i * 7);
  cord_buf b;
  ASSERT_TRUE(SerializeAsCompressedData(m, &b, COMPRESS_TYPE_LZ4));
  ASSERT_TRUE(ParseFromCompressedData(b, &m2, COMPRESS_TYPE_LZ4));
  ASSERT_EQ(m2.text(), m.text());
  ASSERT_EQ(m2.numbers_size(), 3);
  cord_buf bad;
  bad.append(std::string("\x05\x50hel", 5));  // literals cut short
  ASSERT_FALSE(policy::Lz4Decompress(bad, &back));
  // a tiny body whose header claims 0xFFFFFFFF bytes: rejected by the length
  // bound before anything is allocated for it (no bad_alloc out of the handler)
  cord_buf huge;
  huge.append(std::string("\xff\xff\xff\xff\x0f\x10\x61", 7));
  ASSERT_FALSE(policy::Lz4Decompress(huge, &back));
}

TEST_CPU(cord_buf_blocks) {
  cord_buf b;
  std::string s = pattern(20000, true);
  b.append(s);
  ASSERT_EQ(b.size(), s.size());
  ASSERT_EQ(b.backing_block_num(), 3u);  // 8160 + 8160 + 3680
  ASSERT_EQ(b.backing_block(0).size(), cord_buf::kBlockPayload);
  ASSERT_EQ(b.to_string(), s);
  cord_buf head;
  ASSERT_EQ(b.cutn(&head, 9000), 9000u);
  ASSERT_EQ(head.to_string(), s.substr(0, 9000));
  ASSERT_EQ(b.to_string(), s.substr(9000));
  static std::atomic<int> freed{0};
  char* user = (char*)malloc(100);
  memset(user, 'u', 100);
  {
    cord_buf u;
    u.append_user_data(user, 100, [](void* p) { freed++; free(p); });
    cord_buf copy = u;
    ASSERT_TRUE(copy.equals(std::string(100, 'u')));
  }
  ASSERT_EQ(freed.load(), 1);
}

TEST_CPU(cord_buf_append_self) {
  // the reference's append(const cord_buf&) works when other == *this
  cord_buf b;
  std::string s = pattern(30000, true);  // 4 refs: the append below reallocates
  b.append(s);
  b.append(b);
  ASSERT_EQ(b.size(), 2 * s.size());
  ASSERT_EQ(b.to_string(), s + s);
  b.append(b);
  ASSERT_EQ(b.to_string(), s + s + s + s);
}

TEST_CPU(cord_buf_blockmem_hook) {
  static std::atomic<int> allocs{0};
  void* (*old_a)(size_t) = flare::iobuf::blockmem_allocate;
  flare::iobuf::blockmem_allocate = [](size_t n) -> void* { allocs++; return malloc(n); };
  {
    cord_buf b;
    b.append(pattern(17000, false));
  }
  flare::iobuf::blockmem_allocate = old_a;
  ASSERT_EQ(allocs.load(), 3);
}

TEST_CPU(snappy_message_wire_format) {
  snappy_message::SnappyMessageProto m;
  m.set_text("Hello World!");
  m.add_numbers(2);
  m.add_numbers(7);
  m.add_numbers(45);
  m.add_numbers(-1);
  const std::string w = m.SerializeAsString();
  ASSERT_EQ(hex(w), "0a0c48656c6c6f20576f726c642110021007102d10ffffffffffffffffff01");
  snappy_message::SnappyMessageProto p;
  ASSERT_TRUE(p.ParseFromString(w));
  ASSERT_EQ(p.numbers_size(), 4);
  ASSERT_EQ(p.numbers(3), -1);
}

// ------------------------------------------------------------------ GPU tests
// rpc_snappy_compress_test.cc:82-97
TEST_GPU(snappy) {
  snappy_message::SnappyMessageProto old_msg;
  old_msg.set_text("Hello World!");
  old_msg.add_numbers(2);
  old_msg.add_numbers(7);
  old_msg.add_numbers(45);
  cord_buf buf;
  ASSERT_TRUE(policy::SnappyCompress(old_msg, &buf));
  snappy_message::SnappyMessageProto new_msg;
  ASSERT_TRUE(policy::SnappyDecompress(buf, &new_msg));
  ASSERT_TRUE(strcmp(new_msg.text().c_str(), "Hello World!") == 0);
  ASSERT_TRUE(new_msg.numbers_size() == 3);
  ASSERT_EQ(new_msg.numbers(0), 2);
  ASSERT_EQ(new_msg.numbers(1), 7);
  ASSERT_EQ(new_msg.numbers(2), 45);
}

// :99-106, plus the exact bytes the reference emits
TEST_GPU(snappy_iobuf) {
  cord_buf buf, output_buf, check_buf;
  const char* test = "this is a test";
  buf.append(test, strlen(test));
  ASSERT_TRUE(policy::SnappyCompress(buf, &output_buf));
  ASSERT_EQ(hex(output_buf.to_string()), "0e34" + hex(test));
  ASSERT_TRUE(policy::SnappyDecompress(output_buf, &check_buf));
  ASSERT_EQ(check_buf.to_string(), std::string(test));
}

// :108-137
TEST_GPU(mass_snappy) {
  snappy_message::SnappyMessageProto old_msg;
  const std::string text = pattern(12435, true);
  old_msg.set_text(text);
  old_msg.add_numbers(2);
  old_msg.add_numbers(7);
  old_msg.add_numbers(45);
  cord_buf buf;
  ASSERT_TRUE(policy::SnappyCompress(old_msg, &buf));
  snappy_message::SnappyMessageProto new_msg;
  ASSERT_TRUE(policy::SnappyDecompress(buf, &new_msg));
  ASSERT_EQ(new_msg.text(), text);
  ASSERT_EQ(new_msg.numbers_size(), 3);
  ASSERT_EQ(new_msg.numbers(2), 45);
}

// :139-166, plus the known answer for the 200-byte pattern
TEST_GPU(snappy_test) {
  const std::string text = pattern(200, true);
  std::string output, append_string;
  ASSERT_TRUE(flare::snappy::Compress(text.data(), text.size(), &output));
  ASSERT_EQ(hex(output), "c80190" + hex(text.substr(0, 37)) + "fe2400fe24008a2400");
  const size_t com_len1 = output.size();
  ASSERT_TRUE(flare::snappy::Compress("123456", 6, &append_string));
  output.append(append_string);
  std::string u1, u2;
  ASSERT_TRUE(flare::snappy::Uncompress(output.data(), com_len1, &u1));
  ASSERT_EQ(u1, text);
  ASSERT_TRUE(flare::snappy::Uncompress(append_string.data(), append_string.size(), &u2));
  ASSERT_EQ(u2, "123456");
}

// :238-257 (handler compress, flat GetUncompressedLength + RawUncompress)
TEST_GPU(mass_snappy_iobuf) {
  const std::string text = pattern(782, false);
  cord_buf buf, output_buf;
  buf.append(text);
  ASSERT_TRUE(policy::SnappyCompress(buf, &output_buf));
  const std::string out = output_buf.to_string();
  size_t dl = 0;
  ASSERT_TRUE(flare::snappy::GetUncompressedLength(out.data(), out.size(), &dl));
  std::string dec(dl, '\0');
  ASSERT_TRUE(flare::snappy::RawUncompress(out.data(), out.size(), &dec[0]));
  ASSERT_EQ(dec, text);
}

// :168-236 -- prints throughput like the reference; asserts only correctness
TEST_GPU(throughput_compare) {
  const int len_subs[] = {128, 1024, 16 * 1024, 32 * 1024, 512 * 1024};
  printf("%20s%20s%25s%25s\n", "Compress size(B)", "ratio", "Compress MB/s", "Decompress MB/s");
  for (int len : len_subs) {
    snappy_message::SnappyMessageProto old_msg;
    old_msg.set_text(pattern(len, true));
    const int k = std::min(32 * 1024 * 1024 / len, 200);
    size_t clen = 0;
    double tc = 0, td = 0;
    for (int i = 0; i < k; ++i) {
      cord_buf b;
      auto t0 = std::chrono::steady_clock::now();
      ASSERT_TRUE(policy::SnappyCompress(old_msg, &b));
      auto t1 = std::chrono::steady_clock::now();
      snappy_message::SnappyMessageProto m;
      ASSERT_TRUE(policy::SnappyDecompress(b, &m));
      auto t2 = std::chrono::steady_clock::now();
      ASSERT_EQ(m.text().size(), (size_t)len);
      clen += b.size();
      tc += std::chrono::duration<double>(t1 - t0).count();
      td += std::chrono::duration<double>(t2 - t1).count();
    }
    printf("%20d%20.3f%25.1f%25.1f\n", len, (double)clen / k / len, (double)len * k / tc / 1e6,
           (double)len * k / td / 1e6);
  }
}

TEST_GPU(fragmentation_independent) {
  const std::string text = pattern(100000, true) + pattern(30000, false);
  cord_buf whole;
  whole.append(text);
  cord_buf ref_out;
  ASSERT_TRUE(policy::SnappyCompress(whole, &ref_out));
  const std::string expect = ref_out.to_string();
  for (size_t piece : {1ul, 7ul, 4096ul, 8160ul, 65536ul}) {
    cord_buf frag;
    for (size_t p = 0; p < text.size(); p += piece) {
      cord_buf one;
      one.append(text.data() + p, std::min(piece, text.size() - p));
      frag.append(one);  // reference-append: one backing block per piece
    }
    cord_buf out, back;
    ASSERT_TRUE(policy::SnappyCompress(frag, &out));
    ASSERT_EQ(out.to_string(), expect);
    ASSERT_TRUE(policy::SnappyDecompress(out, &back));
    ASSERT_TRUE(back.equals(text));
  }
}

TEST_GPU(corrupt_input_rejected) {
  cord_buf bad, out;
  bad.append(std::string("\x08\x0c" "abcd" "\x01\x00", 8));  // offset 0
  ASSERT_FALSE(policy::SnappyDecompress(bad, &out));
  cord_buf trunc;
  trunc.append(std::string("\x80", 1));
  snappy_message::SnappyMessageProto m;
  ASSERT_FALSE(policy::SnappyDecompress(trunc, &m));
  // lenient 5-byte header accepted by the Source path, rejected by the flat API
  std::string l("\xff\xff\xff\xff\x1f", 5);
  size_t ul = 0;
  ASSERT_FALSE(flare::snappy::GetUncompressedLength(l.data(), l.size(), &ul));
  ASSERT_FALSE(flare::snappy::IsValidCompressedBuffer(l.data(), l.size()));
}

TEST_GPU(concurrent_callers_are_batched) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  const auto before = codec.stats();
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 16; ++t) {
    th.emplace_back([t, &bad] {
      for (int i = 0; i < 50; ++i) {
        snappy_message::SnappyMessageProto m;
        m.set_text(pattern(1000 + 37 * t + i, (i & 1) != 0));
        m.add_numbers(t);
        cord_buf b;
        snappy_message::SnappyMessageProto r;
        if (!policy::SnappyCompress(m, &b) || !policy::SnappyDecompress(b, &r) || r.text() != m.text() ||
            r.numbers(0) != t)
          bad++;
      }
    });
  }
  for (auto& x : th) x.join();
  ASSERT_EQ(bad.load(), 0);
  const auto after = codec.stats();
  ASSERT_EQ(after.messages - before.messages, 1600u);
  printf("  1600 calls in %llu device batches (largest %llu)\n",
         (unsigned long long)(after.batches - before.batches), (unsigned long long)after.max_batch);
  ASSERT_TRUE(after.batches - before.batches < 1600u);  // calls were coalesced
}

TEST_GPU(explicit_batch_api) {
  std::vector<cord_buf> ins(300), comps(300), outs(300);
  std::vector<const cord_buf*> pin;
  std::vector<cord_buf*> pc, po;
  for (int i = 0; i < 300; ++i) {
    ins[i].append(pattern(i * 97 % 70000, i % 3 == 0));
    pin.push_back(&ins[i]);
    pc.push_back(&comps[i]);
    po.push_back(&outs[i]);
  }
  std::vector<bool> ok;
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  ASSERT_TRUE(codec.CompressBatch(pin, pc, &ok));
  std::vector<const cord_buf*> pcc(pc.begin(), pc.end());
  ASSERT_TRUE(codec.UncompressBatch(pcc, po, &ok));
  for (int i = 0; i < 300; ++i) {
    std::string one;
    const std::string s = ins[i].to_string();
    flare::snappy::Compress(s.data(), s.size(), &one);
    ASSERT_EQ(comps[i].to_string(), one);  // batched == single-call bytes
    ASSERT_TRUE(outs[i].equals(s));
  }
}

TEST_GPU(pinned_block_memory) {
  // cord_buf blocks from pinned memory (the blockmem hook, cord_buf.cc:159-166)
  void* (*old_a)(size_t) = flare::iobuf::blockmem_allocate;
  void (*old_d)(void*) = flare::iobuf::blockmem_deallocate;
  flare::iobuf::blockmem_allocate = [](size_t n) -> void* {
    void* p = nullptr;
    return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
  };
  flare::iobuf::blockmem_deallocate = [](void* p) { (void)hipHostFree(p); };
  {
    cord_buf in, out, back;
    in.append(pattern(50000, true));
    ASSERT_TRUE(policy::SnappyCompress(in, &out));
    ASSERT_TRUE(policy::SnappyDecompress(out, &back));
    ASSERT_TRUE(back.equals(in.to_string()));
  }
  flare::iobuf::blockmem_allocate = old_a;
  flare::iobuf::blockmem_deallocate = old_d;
}

// ------------------------------------------------- host runtime (policy) tests
static std::string flat_compress(const std::string& s) {
  std::string o;
  flare::snappy::Compress(s.data(), s.size(), &o);
  return o;
}

TEST_CPU(flat_api_on_host_codec) {
  // no GPU in the CPU run: the flat API runs the host codec; compress never fails
  const std::string t = pattern(200, true);
  std::string c;
  ASSERT_EQ(flare::snappy::Compress(t.data(), t.size(), &c), 49u);
  ASSERT_EQ(hex(c).substr(0, 6), "c80190");  // known answer
  std::string back;
  ASSERT_TRUE(flare::snappy::Uncompress(c.data(), c.size(), &back));
  ASSERT_EQ(back, t);
  ASSERT_TRUE(flare::snappy::IsValidCompressedBuffer(c.data(), c.size()));
  ASSERT_FALSE(flare::snappy::IsValidCompressedBuffer(c.data(), c.size() - 1));
  cord_buf in, out, b2;
  in.append(pattern(70000, false));
  ASSERT_TRUE(policy::SnappyCompress(in, &out));
  ASSERT_EQ(out.to_string(), flat_compress(in.to_string()));
  ASSERT_TRUE(policy::SnappyDecompress(out, &b2));
  ASSERT_TRUE(b2.equals(in.to_string()));
}

TEST_CPU(iovec_and_as_much_as_possible) {
  const std::string t = pattern(5000, true);
  const std::string c = flat_compress(t);
  char a[1000], b[3000], d[2000];
  struct iovec iov[3] = {{a, sizeof(a)}, {b, sizeof(b)}, {d, sizeof(d)}};
  ASSERT_TRUE(flare::snappy::RawUncompressToIOVec(c.data(), c.size(), iov, 3));
  ASSERT_EQ(std::string(a, 1000) + std::string(b, 3000) + std::string(d, 1000), t);
  ASSERT_FALSE(flare::snappy::RawUncompressToIOVec(c.data(), c.size(), iov, 2));  // 4000 < 5000
  // a truncated stream: the scattered writer keeps every complete tag
  cord_buf in, out;
  in.append(c.substr(0, c.size() / 2));
  const size_t r = flare::snappy::UncompressAsMuchAsPossible(in, &out);
  ASSERT_EQ(r, out.size());
  ASSERT_TRUE(out.size() > 0 && out.size() < t.size());
  ASSERT_EQ(out.to_string(), t.substr(0, out.size()));
}

TEST_GPU(threshold_routes_small_bodies_to_host) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  codec.SetMinGpuBytes(16384);
  const auto s0 = codec.stats();
  cord_buf small, big, o1, o2;
  small.append(pattern(4096, true));
  big.append(pattern(65536, false));
  ASSERT_TRUE(policy::SnappyCompress(small, &o1));
  const auto s1 = codec.stats();
  ASSERT_TRUE(policy::SnappyCompress(big, &o2));
  const auto s2 = codec.stats();
  codec.SetMinGpuBytes(0);
  ASSERT_EQ(s1.cpu_messages - s0.cpu_messages, 1u);
  ASSERT_EQ(s1.messages, s0.messages);
  ASSERT_EQ(s2.messages - s1.messages, 1u);
  ASSERT_EQ(o1.to_string(), flat_compress(small.to_string()));  // same bytes either way
  ASSERT_EQ(o2.to_string(), flat_compress(big.to_string()));
}

TEST_GPU(device_error_falls_back_to_host) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  const auto s0 = codec.stats();
  cord_buf in, c, back;
  in.append(pattern(50000, true));
  flare::gpu::InjectDeviceErrorsForTesting(2);
  ASSERT_TRUE(policy::SnappyCompress(in, &c));
  ASSERT_TRUE(policy::SnappyDecompress(c, &back));
  const auto s1 = codec.stats();
  ASSERT_EQ(s1.fallbacks - s0.fallbacks, 2u);
  ASSERT_EQ(c.to_string(), flat_compress(in.to_string()));
  ASSERT_TRUE(back.equals(in.to_string()));
  cord_buf bad, o;
  bad.append(c.to_string().substr(0, c.size() - 7));
  flare::gpu::InjectDeviceErrorsForTesting(1);
  ASSERT_FALSE(policy::SnappyDecompress(bad, &o));  // the host codec's verdict is the reference's
}

TEST_GPU(outputs_adopted_from_pinned_slabs) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  const std::string t = pattern(60000, true);
  cord_buf in, c;
  in.append(t);
  ASSERT_TRUE(policy::SnappyCompress(in, &c));
  for (int i = 0; i < 300; ++i) {  // slabs go back to the pool as outputs die
    const auto s0 = codec.stats();
    cord_buf back;
    ASSERT_TRUE(policy::SnappyDecompress(c, &back));
    ASSERT_EQ(codec.stats().adopted - s0.adopted, 1u);
    ASSERT_EQ(back.backing_block_num(), 1u);
    std::string_view v = back.backing_block(0);
    ASSERT_TRUE(flare::gpu::IsPinned(v.data(), v.size()));
    ASSERT_TRUE(back.equals(t));
  }
}

TEST_GPU(pinned_blocks_read_by_the_gpu) {
  void* (*old_a)(size_t) = flare::iobuf::blockmem_allocate;
  void (*old_d)(void*) = flare::iobuf::blockmem_deallocate;
  ASSERT_EQ(flare::gpu::UsePinnedBlocks(), 0);
  {
    std::vector<cord_buf> ins(40), cs(40), outs(40);
    std::vector<const cord_buf*> pin, pcc;
    std::vector<cord_buf*> pc, po;
    for (int i = 0; i < 40; ++i) {
      ins[i].append(pattern(20000 + 3001 * i, i & 1));
      std::string_view v = ins[i].backing_block(0);
      ASSERT_TRUE(flare::gpu::IsPinned(v.data(), v.size()));
      pin.push_back(&ins[i]);
      pc.push_back(&cs[i]);
      po.push_back(&outs[i]);
    }
    std::vector<bool> ok;
    auto& codec = flare::gpu::SnappyGpuCodec::Instance();
    ASSERT_TRUE(codec.CompressBatch(pin, pc, &ok));
    for (auto* p : pc) pcc.push_back(p);
    ASSERT_TRUE(codec.UncompressBatch(pcc, po, &ok));
    for (int i = 0; i < 40; ++i) {
      ASSERT_EQ(cs[i].to_string(), flat_compress(ins[i].to_string()));
      ASSERT_TRUE(outs[i].equals(ins[i].to_string()));
    }
  }  // every pinned block released before the hooks go back
  flare::iobuf::blockmem_allocate = old_a;
  flare::iobuf::blockmem_deallocate = old_d;
}

namespace {
struct TestLatch {
  std::mutex mu;
  std::condition_variable cv;
  bool set = false;
};
std::atomic<int> g_park[4];
}  // namespace

TEST_GPU(park_hooks_used_by_followers) {
  for (auto& x : g_park) x = 0;
  flare::gpu::ParkHooks h;
  h.create = [] { ++g_park[0]; return (void*)new TestLatch; };
  h.wait = [](void* p) {
    ++g_park[1];
    auto* l = static_cast<TestLatch*>(p);
    std::unique_lock<std::mutex> lk(l->mu);
    l->cv.wait(lk, [&] { return l->set; });
  };
  h.signal = [](void* p) {
    ++g_park[2];
    auto* l = static_cast<TestLatch*>(p);
    std::lock_guard<std::mutex> lk(l->mu);
    l->set = true;
    l->cv.notify_all();
  };
  h.destroy = [](void* p) { ++g_park[3]; delete static_cast<TestLatch*>(p); };
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  codec.SetParkHooks(h);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 16; ++t)
    th.emplace_back([t, &bad] {
      for (int i = 0; i < 40; ++i) {
        cord_buf in, c, back;
        in.append(pattern(20000 + 97 * t + i, true));
        if (!policy::SnappyCompress(in, &c) || !policy::SnappyDecompress(c, &back) ||
            !back.equals(in.to_string()))
          bad++;
      }
    });
  for (auto& x : th) x.join();
  codec.SetParkHooks(flare::gpu::ParkHooks{});
  ASSERT_EQ(bad.load(), 0);
  printf("  latches: %d created, %d waits, %d signals, %d destroyed\n", g_park[0].load(), g_park[1].load(),
         g_park[2].load(), g_park[3].load());
  ASSERT_TRUE(g_park[0].load() > 0);
  ASSERT_EQ(g_park[0].load(), g_park[1].load());
  ASSERT_EQ(g_park[0].load(), g_park[2].load());
  ASSERT_EQ(g_park[0].load(), g_park[3].load());
}

TEST_GPU(device_mask_init_and_shutdown) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  ASSERT_EQ(codec.InitDevices(1), 1);
  codec.Shutdown();
  ASSERT_FALSE(codec.available());
  const auto s0 = codec.stats();
  cord_buf in, c, back;
  in.append(pattern(70000, true));
  ASSERT_TRUE(policy::SnappyCompress(in, &c));  // host codec while shut down
  ASSERT_TRUE(policy::SnappyDecompress(c, &back));
  const auto s1 = codec.stats();
  ASSERT_EQ(s1.messages, s0.messages);
  ASSERT_EQ(s1.cpu_messages - s0.cpu_messages, 2u);
  ASSERT_TRUE(codec.InitDevices(0) >= 1);
  cord_buf c2;
  ASSERT_TRUE(policy::SnappyCompress(in, &c2));
  ASSERT_EQ(codec.stats().messages - s1.messages, 1u);
  ASSERT_EQ(c2.to_string(), c.to_string());
  ASSERT_TRUE(back.equals(in.to_string()));
}

TEST_GPU(validate_only_on_device) {
  auto& codec = flare::gpu::SnappyGpuCodec::Instance();
  const std::string c = flat_compress(pattern(100000, true));
  const auto s0 = codec.stats();
  ASSERT_TRUE(flare::snappy::IsValidCompressedBuffer(c.data(), c.size()));
  ASSERT_FALSE(flare::snappy::IsValidCompressedBuffer(c.data(), c.size() - 1));
  ASSERT_EQ(codec.stats().messages - s0.messages, 2u);
}

int main(int argc, char** argv) {
  bool want_cpu = true, want_gpu = false;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--gpu")) { want_gpu = true; want_cpu = false; }
    if (!strcmp(argv[i], "--all")) { want_gpu = true; want_cpu = true; }
  }
  if (want_gpu) {
    GlobalInitializeSnappyGpu();
    flare::gpu::SnappyGpuCodec::Instance().SetMinGpuBytes(0);  // every body to the GPU
    if (!flare::gpu::SnappyGpuCodec::Instance().available()) {
      fprintf(stderr, "GPU codec unavailable: %s\n", flare::gpu::SnappyGpuCodec::Instance().error().c_str());
      return 2;
    }
  }
  int run = 0;
  for (auto& t : registry()) {
    if ((t.gpu && !want_gpu) || (!t.gpu && !want_cpu)) continue;
    ++run;
    try {
      t.fn();
      printf("[  OK  ] %s\n", t.name);
    } catch (const Failure&) {
      printf("[ FAIL ] %s\n", t.name);
      ++g_failures;
    }
  }
  printf("%d tests, %d failures\n", run, g_failures);
  return g_failures ? 1 : 0;
}

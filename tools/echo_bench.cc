// echo_bench.cc -- BASELINE config 1: example/echo over
// loopback with CompressType=snappy, a 4 KiB request body, one client thread.
//
// Client and server are this repo's baidu_std framing (host/
// baidu_rpc_protocol.*) over a TCP socket on 127.0.0.1, following
// /root/reference/example/echo/{client,server}.cc: the client sets
// set_request_compress_type(SNAPPY) (as test/rpc/rpc_public_prpc_protocol_
// test.cc:272 does), the server echoes EchoRequest.message into
// EchoResponse.message and compresses the response with the request's type.
// EchoRequest.message is 4,093 bytes, so the serialized body is exactly
// 4,096 bytes (0a fd 1f + 4,093).  The client's loop has no sleep (the
// example's -interval_ms) so it measures QPS.
//
//   echo_bench --codec runtime      the drop-in handler (GPU runtime with its
//                                   host codec below the size threshold)
//   echo_bench --codec gpu          the drop-in handler with every body sent
//                                   to the GPU (threshold 0)
//   echo_bench --codec reference    the reference's own Snappy (oracle/_ref,
//                                   loaded only here, for bench.py's
//                                   cpu_baseline leg)
//   echo_bench --codec host         the runtime's host codec called directly
//   echo_bench --codec none         COMPRESS_TYPE_NONE: the transport floor
// Prints one JSON object: calls, QPS, p50/p99/mean latency (us) and the share
// of client+server time spent inside the compress handlers.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <sched.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "baidu_rpc_protocol.h"
#include "compress.h"
#include "cord_buf.h"
#include "gpu_codec.h"
#include "snappy_compress.h"

using namespace flare::rpc;
using flare::cord_buf;

extern "C" void dg_text_body(uint64_t index, uint8_t* out, size_t n);

namespace {

// example/echo/echo.proto: message EchoRequest/EchoResponse { required string message = 1; }
class EchoMessage : public Message {
 public:
  std::string message;
  bool has = false;
  bool SerializeToCordBuf(cord_buf* out) const override {
    if (!has) return false;  // a required field is missing
    std::string s;
    s.push_back('\x0a');
    uint64_t v = message.size();
    while (v >= 128) {
      s.push_back((char)(v | 128));
      v >>= 7;
    }
    s.push_back((char)v);
    s += message;
    out->append(s);
    return true;
  }
  bool ParseFromCordBuf(const cord_buf& in) override {
    const std::string s = in.to_string();
    size_t p = 0;
    has = false;
    while (p < s.size()) {
      uint64_t key = 0, len = 0;
      for (int sh = 0; p < s.size(); sh += 7) {
        const uint8_t b = (uint8_t)s[p++];
        key |= (uint64_t)(b & 127) << sh;
        if (b < 128) break;
      }
      if (key != 0x0a) return false;
      for (int sh = 0; p < s.size(); sh += 7) {
        const uint8_t b = (uint8_t)s[p++];
        len |= (uint64_t)(b & 127) << sh;
        if (b < 128) break;
      }
      if (len > s.size() - p) return false;
      message.assign(s, p, len);
      has = true;
      p += len;
    }
    return has;  // required
  }
};

// ---- codec time accounting: the registered handler wraps the chosen one
std::atomic<uint64_t> g_codec_ns{0};
bool (*g_comp)(const Message&, cord_buf*) = nullptr;
bool (*g_decomp)(const cord_buf&, Message*) = nullptr;

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
bool timed_compress(const Message& m, cord_buf* b) {
  const uint64_t t = now_ns();
  const bool r = g_comp(m, b);
  g_codec_ns += now_ns() - t;
  return r;
}
bool timed_decompress(const cord_buf& d, Message* m) {
  const uint64_t t = now_ns();
  const bool r = g_decomp(d, m);
  g_codec_ns += now_ns() - t;
  return r;
}

// ---- the reference's Snappy (oracle/_ref/libsnappy_ref.so, baseline only)
size_t (*ref_compress)(const char*, size_t, char*, size_t) = nullptr;
size_t (*ref_max)(size_t) = nullptr;
int (*ref_uncompress)(const char*, size_t, char*, size_t, size_t*, size_t) = nullptr;
int (*ref_len)(const char*, size_t, uint32_t*) = nullptr;

bool ref_snappy_compress(const Message& m, cord_buf* buf) {
  cord_buf pb;
  if (!m.SerializeToCordBuf(&pb)) return false;
  const std::string s = pb.to_string();
  std::string out(ref_max(s.size()), '\0');
  out.resize(ref_compress(s.data(), s.size(), &out[0], 8160));
  buf->append(out);
  return true;
}
bool ref_snappy_decompress(const cord_buf& data, Message* m) {
  const std::string s = data.to_string();
  uint32_t ul = 0;
  if (!ref_len(s.data(), s.size(), &ul)) return false;
  std::string out(ul, '\0');
  size_t prod = 0;
  if (!ref_uncompress(s.data(), s.size(), &out[0], ul, &prod, 8160)) return false;
  cord_buf b;
  b.append(out);
  return m->ParseFromCordBuf(b);
}

bool write_all(int fd, const cord_buf& b) {
  for (size_t i = 0; i < b.backing_block_num(); ++i) {
    std::string_view v = b.backing_block(i);
    size_t off = 0;
    while (off < v.size()) {
      const ssize_t k = ::send(fd, v.data() + off, v.size() - off, MSG_NOSIGNAL);
      if (k <= 0) return false;
      off += (size_t)k;
    }
  }
  return true;
}

// Reads until one whole frame can be cut from `rbuf`.
bool read_frame(int fd, cord_buf* rbuf, MostCommonMessage* msg) {
  char tmp[65536];
  for (;;) {
    const ParseError e = policy::ParseRpcMessage(rbuf, msg);
    if (e == PARSE_OK) return true;
    if (e != PARSE_ERROR_NOT_ENOUGH_DATA) return false;
    const ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
    if (k <= 0) return false;
    rbuf->append(tmp, (size_t)k);
  }
}

void server(int lfd, std::atomic<bool>* bad) {
  const int fd = ::accept(lfd, nullptr, nullptr);
  if (fd < 0) {
    *bad = true;
    return;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  cord_buf rbuf;
  for (;;) {
    MostCommonMessage msg;
    if (!read_frame(fd, &rbuf, &msg)) break;  // client closed
    Controller cntl;
    EchoMessage req;
    policy::RpcMeta meta;
    if (!policy::ProcessRpcRequest(&msg, &cntl, &req, &meta)) {
      *bad = true;
      break;
    }
    EchoMessage res;
    res.message = req.message;  // example/echo/server.cc: response->set_message(request->message())
    res.has = true;
    cntl.set_response_compress_type(cntl.request_compress_type());
    cord_buf out;
    policy::SendRpcResponse(meta.correlation_id(), &cntl, &res, &out);
    if (!write_all(fd, out)) break;
  }
  ::close(fd);
}

}  // namespace

int main(int argc, char** argv) {
  std::string codec = "runtime";
  int calls = 20000, warmup = 500;
  size_t msg_len = 4093;
  for (int i = 1; i + 1 < argc; ++i) {
    if (!strcmp(argv[i], "--codec")) codec = argv[i + 1];
    if (!strcmp(argv[i], "--calls")) calls = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--warmup")) warmup = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--message-bytes")) msg_len = (size_t)atol(argv[i + 1]);
  }
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--init-hip")) {  // diagnostic: HIP runtime up, unused
      cpu_set_t a0, a1;
      sched_getaffinity(0, sizeof(a0), &a0);
      int n = 0;
      (void)hipGetDeviceCount(&n);
      sched_getaffinity(0, sizeof(a1), &a1);
      fprintf(stderr, "affinity cpus before %d after %d\n", CPU_COUNT(&a0), CPU_COUNT(&a1));
    }
  CompressType type = COMPRESS_TYPE_SNAPPY;
  if (codec == "runtime" || codec == "gpu") {
    GlobalInitializeSnappyGpu();  // the drop-in: global.cc:372-376's registration
    if (codec == "gpu") flare::gpu::SnappyGpuCodec::Instance().SetMinGpuBytes(0);
    // re-register through the timing wrapper
    const CompressHandler* h = FindCompressHandler(COMPRESS_TYPE_SNAPPY);
    g_comp = h->Compress;
    g_decomp = h->Decompress;
    ResetCompressHandlersForTesting();
  } else if (codec == "host") {
    // the runtime's host codec called directly (no runtime dispatch)
    g_comp = [](const Message& m, cord_buf* b) {
      cord_buf pb;
      return m.SerializeToCordBuf(&pb) && flare::gpu::CpuCompress(pb, b);
    };
    g_decomp = [](const cord_buf& d, Message* m) {
      cord_buf pb;
      return flare::gpu::CpuUncompress(d, &pb) && m->ParseFromCordBuf(pb);
    };
  } else if (codec == "reference") {
    const char* path = getenv("FLARE_SNAPPY_REF_LIB");
    void* L = dlopen(path ? path : "oracle/_ref/libsnappy_ref.so", RTLD_NOW);
    if (!L) {
      fprintf(stderr, "reference library: %s\n", dlerror());
      return 2;
    }
    ref_compress = (decltype(ref_compress))dlsym(L, "ref_compress");
    ref_max = (decltype(ref_max))dlsym(L, "ref_max_compressed_length");
    ref_uncompress = (decltype(ref_uncompress))dlsym(L, "ref_uncompress");
    ref_len = (decltype(ref_len))dlsym(L, "ref_get_uncompressed_length_source");
    if (!ref_compress || !ref_max || !ref_uncompress || !ref_len) return 2;
    g_comp = ref_snappy_compress;
    g_decomp = ref_snappy_decompress;
  } else if (codec == "none") {
    type = COMPRESS_TYPE_NONE;
  } else {
    fprintf(stderr, "unknown --codec %s\n", codec.c_str());
    return 2;
  }
  if (type == COMPRESS_TYPE_SNAPPY &&
      RegisterCompressHandler(COMPRESS_TYPE_SNAPPY, CompressHandler{timed_compress, timed_decompress, "snappy"}) != 0)
    return 2;

  // ---- loopback server
  const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  addr.sin_port = 0;
  socklen_t alen = sizeof(addr);
  if (::bind(lfd, (sockaddr*)&addr, sizeof(addr)) != 0 || ::listen(lfd, 1) != 0 ||
      ::getsockname(lfd, (sockaddr*)&addr, &alen) != 0) {
    perror("listen");
    return 2;
  }
  std::atomic<bool> bad{false};
  std::thread srv(server, lfd, &bad);

  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (::connect(fd, (sockaddr*)&addr, sizeof(addr)) != 0) {
    perror("connect");
    return 2;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));

  EchoMessage req;
  req.message.resize(msg_len);
  dg_text_body(0, reinterpret_cast<uint8_t*>(&req.message[0]), msg_len);  // SURVEY §8(d) text generator
  req.has = true;
  size_t body_bytes = 0;
  {
    cord_buf b;
    req.SerializeToCordBuf(&b);
    body_bytes = b.size();
  }
  std::vector<double> lat;
  lat.reserve(calls);
  cord_buf rbuf;
  uint64_t codec0 = 0, t0 = 0;
  int errors = 0;
  for (int i = 0; i < warmup + calls; ++i) {
    if (i == warmup) {
      codec0 = g_codec_ns.load();
      t0 = now_ns();
    }
    const uint64_t a = now_ns();
    Controller cntl;
    cntl.set_request_compress_type(type);
    cord_buf body, frame;
    SerializeRequestDefault(&body, &cntl, &req);
    if (cntl.Failed()) return 3;
    policy::PackRpcRequest(&frame, (uint64_t)i + 1, "example.EchoService", "Echo", &cntl, body);
    if (!write_all(fd, frame)) return 3;
    MostCommonMessage msg;
    if (!read_frame(fd, &rbuf, &msg)) return 3;
    EchoMessage res;
    policy::ProcessRpcResponse(&msg, &cntl, &res);
    if (cntl.Failed() || res.message != req.message) ++errors;
    if (i >= warmup) lat.push_back((double)(now_ns() - a) / 1e3);
  }
  const double total_s = (double)(now_ns() - t0) / 1e9;
  const double codec_s = (double)(g_codec_ns.load() - codec0) / 1e9;
  ::shutdown(fd, SHUT_RDWR);
  ::close(fd);
  srv.join();
  ::close(lfd);
  std::vector<double> s = lat;
  std::sort(s.begin(), s.end());
  auto pct = [&](double q) { return s.empty() ? 0.0 : s[std::min(s.size() - 1, (size_t)(q * s.size()))]; };
  double mean = 0;
  for (double x : s) mean += x;
  mean /= std::max<size_t>(1, s.size());
  const auto st = flare::gpu::SnappyGpuCodec::Instance().stats();
  printf("{\"codec\": \"%s\", \"calls\": %d, \"message_bytes\": %zu, \"body_bytes\": %zu, \"qps\": %.1f, "
         "\"p50_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f, \"codec_share\": %.4f, \"errors\": %d, "
         "\"gpu_messages\": %llu, \"host_messages\": %llu, \"server_ok\": %s}\n",
         codec.c_str(), calls, msg_len, body_bytes, calls / total_s, pct(0.5), pct(0.99), mean,
         total_s > 0 ? codec_s / total_s : 0.0, errors, (unsigned long long)st.messages,
         (unsigned long long)st.cpu_messages, bad.load() ? "false" : "true");
  return errors || bad.load() ? 1 : 0;
}

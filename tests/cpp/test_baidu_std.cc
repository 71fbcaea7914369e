// test_baidu_std.cc -- baidu_std framing and rpc_dump capture around the GPU
// snappy handler, and the other protocols' compress-type mappings (SURVEY.md
// §8(f) rows 2-4).
//   ./test_baidu_std --cpu                 framing / meta / dump tests (no GPU)
//   ./test_baidu_std --gpu                 compressed request/response round
//                                          trips and batch frame decode (MI355X)
//   ./test_baidu_std --emit DIR            write the RpcMeta / RpcDumpMeta
//                                          fixtures of kMetaCases to DIR
//   ./test_baidu_std --parse-meta FILE     parse FILE as RpcMeta, print JSON
//   ./test_baidu_std --parse-dump-meta FILE  same for RpcDumpMeta
// The --emit / --parse modes let tests/test_framing.py check the hand-written
// wire format against the pure-Python protobuf runtime in both directions.
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

#include "baidu_rpc_meta.h"
#include "baidu_rpc_protocol.h"
#include "compress.h"
#include "cord_buf.h"
#include "gpu_codec.h"
#include "protocol_compress.h"
#include "rpc_dump.h"
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
struct Failure {};
}  // namespace

#define TEST_CPU(name) static void name(); static Reg reg_##name(#name, false, name); static void name()
#define TEST_GPU(name) static void name(); static Reg reg_##name(#name, true, name); static void name()
#define ASSERT_TRUE(c)                                                              \
  do {                                                                              \
    if (!(c)) {                                                                     \
      fprintf(stderr, "  %s:%d: ASSERT_TRUE(%s) failed\n", __FILE__, __LINE__, #c); \
      throw Failure{};                                                              \
    }                                                                               \
  } while (0)
#define ASSERT_FALSE(c) ASSERT_TRUE(!(c))
#define ASSERT_EQ(a, b) ASSERT_TRUE((a) == (b))

using flare::cord_buf;
using namespace flare::rpc;
using namespace flare::rpc::policy;
using snappy_message::SnappyMessageProto;

static std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : s) {
    o.push_back(d[c >> 4]);
    o.push_back(d[c & 15]);
  }
  return o;
}

static std::string text(size_t n, uint64_t seed) {  // compressible filler
  static const char* words[] = {"flare ", "rpc ", "snappy ", "baidu_std ", "frame ", "meta ", "gpu "};
  std::string t;
  uint64_t s = seed;
  while (t.size() < n) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    t += words[(s >> 33) % 7];
  }
  t.resize(n);
  return t;
}

// ------------------------------------------------------------ meta fixtures
// Shared with tests/test_framing.py (same values, same order).
static std::vector<RpcMeta> meta_cases() {
  std::vector<RpcMeta> v;
  {  // a client request
    RpcMeta m;
    m.mutable_request()->set_service_name("example.EchoService");
    m.mutable_request()->set_method_name("Echo");
    m.mutable_request()->set_log_id(123456789012345ll);
    m.set_compress_type(COMPRESS_TYPE_SNAPPY);
    m.set_correlation_id(42);
    m.set_attachment_size(5);
    v.push_back(m);
  }
  {  // a failed response
    RpcMeta m;
    m.mutable_response()->set_error_code(EREQUEST);
    m.mutable_response()->set_error_text("Fail to parse request message, CompressType=snappy");
    m.set_correlation_id(-7);
    m.set_compress_type(COMPRESS_TYPE_SNAPPY);
    v.push_back(m);
  }
  {  // every field, negative int32 / int64 values, empty strings
    RpcMeta m;
    RpcRequestMeta* r = m.mutable_request();
    r->set_service_name("");
    r->set_method_name("M");
    r->set_log_id(-1);
    r->set_trace_id(1ll << 62);
    r->set_span_id(0);
    r->set_parent_span_id(-(1ll << 40));
    r->set_request_id("x-request-id");
    m.mutable_response()->set_error_code(-1);
    m.set_compress_type(-2);
    m.set_correlation_id(9223372036854775807ll);
    m.set_attachment_size(0);
    m.mutable_chunk_info()->set_stream_id(3);
    m.mutable_chunk_info()->set_chunk_id(4);
    m.set_authentication_data(std::string("\0\xff\x80token", 8));
    m.mutable_stream_settings()->set_stream_id(77);
    m.mutable_stream_settings()->set_need_feedback(true);
    m.mutable_stream_settings()->set_writable(false);
    v.push_back(m);
  }
  {  // empty meta
    v.push_back(RpcMeta());
  }
  return v;
}

static std::vector<RpcDumpMeta> dump_meta_cases() {
  std::vector<RpcDumpMeta> v;
  {
    RpcDumpMeta m;
    m.set_service_name("example.EchoService");
    m.set_method_name("Echo");
    m.set_compress_type(COMPRESS_TYPE_SNAPPY);
    m.set_protocol_type(PROTOCOL_BAIDU_STD);
    m.set_attachment_size(3);
    m.set_authentication_data("auth");
    v.push_back(m);
  }
  {
    RpcDumpMeta m;
    m.set_method_index(-3);
    m.set_compress_type(COMPRESS_TYPE_NONE);
    m.set_protocol_type(PROTOCOL_HULU_PBRPC);
    m.set_user_data(std::string("\x01\x00\x02", 3));
    v.push_back(m);
  }
  return v;
}

static std::string json_str(const std::string& s) { return "\"" + hex(s) + "\""; }

static std::string to_json(const RpcMeta& m) {
  std::ostringstream o;
  o << "{";
  bool first = true;
  auto key = [&](const char* k) {
    if (!first) o << ",";
    first = false;
    o << "\"" << k << "\":";
  };
  if (m.has_request()) {
    const RpcRequestMeta& r = m.request();
    key("request");
    o << "{";
    bool f2 = true;
    auto k2 = [&](const char* k) {
      if (!f2) o << ",";
      f2 = false;
      o << "\"" << k << "\":";
    };
    if (r.has_service_name()) { k2("service_name"); o << json_str(r.service_name()); }
    if (r.has_method_name()) { k2("method_name"); o << json_str(r.method_name()); }
    if (r.has_log_id()) { k2("log_id"); o << r.log_id(); }
    if (r.has_trace_id()) { k2("trace_id"); o << r.trace_id(); }
    if (r.has_span_id()) { k2("span_id"); o << r.span_id(); }
    if (r.has_parent_span_id()) { k2("parent_span_id"); o << r.parent_span_id(); }
    if (r.has_request_id()) { k2("request_id"); o << json_str(r.request_id()); }
    o << "}";
  }
  if (m.has_response()) {
    key("response");
    o << "{";
    bool f2 = true;
    if (m.response().has_error_code()) { o << "\"error_code\":" << m.response().error_code(); f2 = false; }
    if (m.response().has_error_text()) {
      if (!f2) o << ",";
      o << "\"error_text\":" << json_str(m.response().error_text());
    }
    o << "}";
  }
  if (m.has_compress_type()) { key("compress_type"); o << m.compress_type(); }
  if (m.has_correlation_id()) { key("correlation_id"); o << m.correlation_id(); }
  if (m.has_attachment_size()) { key("attachment_size"); o << m.attachment_size(); }
  if (m.has_chunk_info()) {
    key("chunk_info");
    o << "{\"stream_id\":" << m.chunk_info().stream_id() << ",\"chunk_id\":" << m.chunk_info().chunk_id() << "}";
  }
  if (m.has_authentication_data()) { key("authentication_data"); o << json_str(m.authentication_data()); }
  if (m.has_stream_settings()) {
    const flare::rpc::StreamSettings& s = m.stream_settings();
    key("stream_settings");
    o << "{\"stream_id\":" << s.stream_id();
    if (s.has_need_feedback()) o << ",\"need_feedback\":" << (s.need_feedback() ? "true" : "false");
    if (s.has_writable()) o << ",\"writable\":" << (s.writable() ? "true" : "false");
    o << "}";
  }
  o << "}";
  return o.str();
}

static std::string to_json(const RpcDumpMeta& m) {
  std::ostringstream o;
  o << "{";
  bool first = true;
  auto key = [&](const char* k) {
    if (!first) o << ",";
    first = false;
    o << "\"" << k << "\":";
  };
  if (m.has_service_name()) { key("service_name"); o << json_str(m.service_name()); }
  if (m.has_method_name()) { key("method_name"); o << json_str(m.method_name()); }
  if (m.has_method_index()) { key("method_index"); o << m.method_index(); }
  if (m.has_compress_type()) { key("compress_type"); o << m.compress_type(); }
  if (m.has_protocol_type()) { key("protocol_type"); o << m.protocol_type(); }
  if (m.has_attachment_size()) { key("attachment_size"); o << m.attachment_size(); }
  if (m.has_authentication_data()) { key("authentication_data"); o << json_str(m.authentication_data()); }
  if (m.has_user_data()) { key("user_data"); o << json_str(m.user_data()); }
  o << "}";
  return o.str();
}

static std::string read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// ---------------------------------------------------------------- CPU tests
TEST_CPU(header_is_prpc_big_endian) {
  char h[12];
  PackRpcHeader(h, 0x0102, 0x030405);
  ASSERT_EQ(hex(std::string(h, 12)), "50525043" "00030507" "00000102");
}

TEST_CPU(meta_known_bytes) {
  RpcMeta m;
  m.mutable_request()->set_service_name("S");
  m.mutable_request()->set_method_name("M");
  m.set_compress_type(1);
  m.set_correlation_id(300);
  // 0a 06 (0a 01 'S' 12 01 'M') 18 01 20 ac 02
  ASSERT_EQ(hex(m.SerializeAsString()), "0a060a015312014d180120ac02");
  RpcMeta neg;
  neg.set_compress_type(-1);  // int32 -1: 10-byte varint
  ASSERT_EQ(hex(neg.SerializeAsString()), "18ffffffffffffffffff01");
}

TEST_CPU(meta_round_trip_and_required_fields) {
  for (const RpcMeta& m : meta_cases()) {
    RpcMeta p;
    ASSERT_TRUE(p.Parse(m.SerializeAsString()));
    ASSERT_EQ(p.SerializeAsString(), m.SerializeAsString());
    ASSERT_EQ(to_json(p), to_json(m));
  }
  RpcMeta m;
  m.mutable_request()->set_service_name("S");  // method_name (required) missing
  RpcMeta p;
  ASSERT_FALSE(p.Parse(m.SerializeAsString()));
  RpcMeta c;
  c.mutable_chunk_info()->set_stream_id(1);  // chunk_id (required) missing
  ASSERT_FALSE(p.Parse(c.SerializeAsString()));
  // truncated, bad varint, field 0, unknown fields skipped, group rejected
  const std::string good = meta_cases()[0].SerializeAsString();
  ASSERT_FALSE(p.Parse(good.substr(0, good.size() - 1)));
  ASSERT_FALSE(p.Parse(std::string("\x18\xff", 2)));
  ASSERT_FALSE(p.Parse(std::string("\x00\x01", 2)));
  ASSERT_TRUE(p.Parse(std::string("\x48\x05\x52\x02hi\x5d\x01\x02\x03\x04\x61", 12) +
                      std::string(8, '\x09')));
  ASSERT_EQ(to_json(p), "{}");
  // a known field with another wire type is an unknown field
  ASSERT_TRUE(p.Parse(std::string("\x1a\x01\x07", 3)));
  ASSERT_FALSE(p.has_compress_type());
  // last value wins; sub-messages merge
  ASSERT_TRUE(p.Parse(std::string("\x18\x01\x18\x02\x12\x02\x08\x05\x12\x03\x12\x01z", 13)));
  ASSERT_EQ(p.compress_type(), 2);
  ASSERT_EQ(p.response().error_code(), 5);
  ASSERT_EQ(p.response().error_text(), "z");
}

TEST_CPU(dump_meta_closed_enums) {
  RpcDumpMeta d;
  ASSERT_TRUE(d.Parse(std::string("\x20\x07\x28\x01", 4)));  // compress_type 7: not in the enum
  ASSERT_FALSE(d.has_compress_type());
  ASSERT_TRUE(d.has_protocol_type());
  for (const RpcDumpMeta& m : dump_meta_cases()) {
    RpcDumpMeta p;
    ASSERT_TRUE(p.Parse(m.SerializeAsString()));
    ASSERT_EQ(to_json(p), to_json(m));
  }
}

static cord_buf frame_of(const RpcMeta& meta, const std::string& payload) {
  cord_buf b;
  SerializeRpcHeaderAndMeta(&b, meta, payload.size());
  b.append(payload);
  return b;
}

TEST_CPU(parse_rpc_message_errors) {
  MostCommonMessage msg;
  cord_buf src;
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_NOT_ENOUGH_DATA);  // empty
  src.append("PR", 2);
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_NOT_ENOUGH_DATA);  // prefix of the magic
  src.clear();
  src.append("PX", 2);
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_TRY_OTHERS);
  src.clear();
  src.append("HTTP/1.1 200", 12);
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_TRY_OTHERS);
  src.clear();
  src.append("PRPC\0\0\0", 7);
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_NOT_ENOUGH_DATA);  // short header
  // body not complete yet
  RpcMeta meta;
  meta.set_correlation_id(1);
  cord_buf full = frame_of(meta, "payload");
  src.clear();
  src.append(full.to_string().substr(0, full.size() - 1));
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_NOT_ENOUGH_DATA);
  ASSERT_EQ(src.size(), full.size() - 1);  // nothing consumed
  // too big
  const uint64_t saved = FLAGS_max_body_size;
  FLAGS_max_body_size = 6;
  src = frame_of(meta, "payload");
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_TOO_BIG_DATA);
  FLAGS_max_body_size = saved;
  // meta_size > body_size: the frame is popped, TRY_OTHERS
  char h[12];
  PackRpcHeader(h, 9, 0);
  h[11] = 10;  // meta_size 10 > body_size 9
  src.clear();
  src.append(h, 12);
  src.append(std::string(9, 'x'));
  src.append("tail", 4);
  ASSERT_EQ(ParseRpcMessage(&src, &msg), PARSE_ERROR_TRY_OTHERS);
  ASSERT_EQ(src.to_string(), "tail");
}

TEST_CPU(parse_rpc_message_cuts_frames) {
  RpcMeta a, b;
  a.set_correlation_id(1);
  b.set_correlation_id(2);
  cord_buf src = frame_of(a, "first");
  src.append(frame_of(b, ""));
  src.append("PRP", 3);
  MostCommonMessage m1, m2, m3;
  ASSERT_EQ(ParseRpcMessage(&src, &m1), PARSE_OK);
  ASSERT_EQ(m1.meta.to_string(), a.SerializeAsString());
  ASSERT_EQ(m1.payload.to_string(), "first");
  ASSERT_EQ(ParseRpcMessage(&src, &m2), PARSE_OK);
  ASSERT_EQ(m2.payload.size(), 0u);
  ASSERT_EQ(ParseRpcMessage(&src, &m3), PARSE_ERROR_NOT_ENOUGH_DATA);
  ASSERT_EQ(src.to_string(), "PRP");
}

TEST_CPU(uncompressed_request_response_round_trip) {
  // client packs, server processes, server responds, client processes
  SnappyMessageProto req, res, got_req, got_res;
  req.set_text("Hello World!");
  req.add_numbers(2);
  req.add_numbers(-7);
  Controller cc;
  cc.set_log_id(99);
  cc.set_request_id("rid");
  cc.request_attachment().append("ATTACH", 6);
  cord_buf body;
  SerializeRequestDefault(&body, &cc, &req);
  ASSERT_FALSE(cc.Failed());
  cord_buf wire;
  PackRpcRequest(&wire, 1234, "example.EchoService", "Echo", &cc, body);
  MostCommonMessage msg;
  ASSERT_EQ(ParseRpcMessage(&wire, &msg), PARSE_OK);
  Controller sc;
  RpcMeta meta;
  ASSERT_TRUE(ProcessRpcRequest(&msg, &sc, &got_req, &meta));
  ASSERT_FALSE(sc.Failed());
  ASSERT_EQ(got_req.SerializeAsString(), req.SerializeAsString());
  ASSERT_EQ(sc.request_attachment().to_string(), "ATTACH");
  ASSERT_EQ(sc.log_id(), 99);
  ASSERT_EQ(sc.request_id(), "rid");
  ASSERT_EQ(meta.request().service_name(), "example.EchoService");
  ASSERT_EQ(meta.correlation_id(), 1234);
  ASSERT_EQ(meta.attachment_size(), 6);

  res.set_text("pong");
  sc.response_attachment().append("RA", 2);
  cord_buf out;
  SendRpcResponse(meta.correlation_id(), &sc, &res, &out);
  MostCommonMessage rmsg;
  ASSERT_EQ(ParseRpcMessage(&out, &rmsg), PARSE_OK);
  Controller cc2;
  ProcessRpcResponse(&rmsg, &cc2, &got_res);
  ASSERT_FALSE(cc2.Failed());
  ASSERT_EQ(got_res.text(), "pong");
  ASSERT_EQ(cc2.response_attachment().to_string(), "RA");
}

TEST_CPU(request_errors_land_on_controller) {
  // attachment larger than the payload
  RpcMeta meta;
  meta.mutable_request()->set_service_name("S");
  meta.mutable_request()->set_method_name("M");
  meta.set_attachment_size(100);
  cord_buf wire = frame_of(meta, "short");
  MostCommonMessage msg;
  ASSERT_EQ(ParseRpcMessage(&wire, &msg), PARSE_OK);
  Controller sc;
  SnappyMessageProto req;
  ASSERT_TRUE(ProcessRpcRequest(&msg, &sc, &req, nullptr));
  ASSERT_EQ(sc.ErrorCode(), EREQUEST);
  ASSERT_EQ(sc.ErrorText(), "attachment_size=100 is larger than request_size=5");
  // unparsable meta: false (the reference fails the socket)
  MostCommonMessage bad;
  bad.meta.append("\x0a\x05", 2);
  Controller sc2;
  ASSERT_FALSE(ProcessRpcRequest(&bad, &sc2, &req, nullptr));
  // a failed server controller sends error code/text and no body
  Controller f;
  f.SetFailed(-1, "boom");
  SnappyMessageProto res;
  res.set_text("unused");
  cord_buf out;
  SendRpcResponse(5, &f, &res, &out);
  MostCommonMessage rmsg;
  ASSERT_EQ(ParseRpcMessage(&out, &rmsg), PARSE_OK);
  ASSERT_EQ(rmsg.payload.size(), 0u);
  Controller cc;
  SnappyMessageProto got;
  ProcessRpcResponse(&rmsg, &cc, &got);
  ASSERT_EQ(cc.ErrorCode(), EINTERNAL);  // -1 is replaced by EINTERNAL
  ASSERT_EQ(cc.ErrorText(), "boom");
}

static std::string tmpdir(const char* tag) {
  char buf[256];
  snprintf(buf, sizeof(buf), "/tmp/fsg_dump_%s_%d", tag, (int)getpid());
  std::string cmd = std::string("rm -rf ") + buf;
  (void)!system(cmd.c_str());
  return buf;
}

TEST_CPU(rpc_dump_serialize_pop) {
  SampledRequest s;
  s.meta = dump_meta_cases()[0];
  s.request.append("compressed-bytes+att", 20);
  cord_buf buf;
  ASSERT_TRUE(SerializeSample(&buf, s));
  const std::string wire = buf.to_string();
  ASSERT_EQ(wire.substr(0, 4), "PRPC");
  bool err = false;
  cord_buf partial;
  partial.append(wire.substr(0, wire.size() - 1));
  ASSERT_TRUE(SampleIterator::Pop(partial, &err) == nullptr);
  ASSERT_FALSE(err);
  auto p = SampleIterator::Pop(buf, &err);
  ASSERT_TRUE(p != nullptr);
  ASSERT_EQ(to_json(p->meta), to_json(s.meta));
  ASSERT_EQ(p->request.to_string(), "compressed-bytes+att");
  ASSERT_EQ(buf.size(), 0u);
  cord_buf bad;
  bad.append("XRPC" + std::string(8, '\0'));
  ASSERT_TRUE(SampleIterator::Pop(bad, &err) == nullptr);
  ASSERT_TRUE(err);
  err = false;
  cord_buf badmeta;
  char h[12];
  PackRpcHeader(h, 2, 0);
  badmeta.append(h, 12);
  badmeta.append("\x0a\x09", 2);  // string longer than the meta
  ASSERT_TRUE(SampleIterator::Pop(badmeta, &err) == nullptr);
  ASSERT_TRUE(err);
}

TEST_CPU(rpc_dump_writer_and_iterator) {
  const std::string dir = tmpdir("w");
  std::vector<std::string> expect;
  {
    RpcDumpWriter w(dir, /*max_requests_in_one_file=*/3, /*max_files=*/32);
    for (int i = 0; i < 8; ++i) {
      SampledRequest s;
      s.meta.set_service_name("svc");
      s.meta.set_method_name("m" + std::to_string(i));
      s.meta.set_compress_type(COMPRESS_TYPE_NONE);
      s.request.append(text(100 + 997 * i, i));
      expect.push_back(s.request.to_string());
      ASSERT_TRUE(w.Dump(s));
    }
    ASSERT_TRUE(w.Flush());
    ASSERT_EQ(w.files().size(), 3u);  // 3 + 3 + 2
  }
  SampleIterator it(dir);
  size_t k = 0;
  while (auto s = it.Next()) {
    ASSERT_TRUE(k < expect.size());
    ASSERT_EQ(s->meta.method_name(), "m" + std::to_string(k));
    ASSERT_EQ(s->request.to_string(), expect[k]);
    ++k;
  }
  ASSERT_EQ(k, expect.size());
  // max_files: the oldest files are removed
  const std::string dir2 = tmpdir("rot");
  RpcDumpWriter w2(dir2, 1, 2);
  for (int i = 0; i < 5; ++i) {
    SampledRequest s;
    s.meta.set_method_name("r" + std::to_string(i));
    s.request.append("x", 1);
    ASSERT_TRUE(w2.Dump(s));
  }
  ASSERT_EQ(w2.files().size(), 2u);
  SampleIterator it2(dir2);
  auto a = it2.Next();
  auto b = it2.Next();
  ASSERT_TRUE(a && b && !it2.Next());
  ASSERT_EQ(a->meta.method_name(), "r3");
  ASSERT_EQ(b->meta.method_name(), "r4");
}

TEST_CPU(rpc_dump_iterator_skips_bad_file) {
  const std::string dir = tmpdir("bad");
  {
    RpcDumpWriter w(dir, 2, 8);
    for (int i = 0; i < 4; ++i) {
      SampledRequest s;
      s.meta.set_method_name("g" + std::to_string(i));
      s.request.append("body", 4);
      w.Dump(s);
    }
  }
  // a garbage file (sorts first) is abandoned at its first frame
  FILE* f = fopen((dir + "/requests.0_garbage").c_str(), "wb");
  fwrite("NOPE-NOT-A-FRAME", 1, 16, f);
  fclose(f);
  SampleIterator it(dir);
  std::vector<std::string> names;
  while (auto s = it.Next()) names.push_back(s->meta.method_name());
  ASSERT_EQ(names.size(), 4u);  // the garbage file yields nothing
  ASSERT_EQ(names[0], "g0");
  ASSERT_EQ(names[3], "g3");
}

TEST_CPU(replay_frame_from_sample) {
  SampledRequest s;
  s.meta.set_service_name("example.EchoService");
  s.meta.set_method_name("Echo");
  s.meta.set_compress_type(COMPRESS_TYPE_SNAPPY);
  s.meta.set_attachment_size(3);
  s.request.append("zzzzzzATT", 9);
  cord_buf frame;
  ReplayAsBaiduStd(s, 77, &frame);
  MostCommonMessage msg;
  ASSERT_EQ(ParseRpcMessage(&frame, &msg), PARSE_OK);
  RpcMeta meta;
  ASSERT_TRUE(meta.Parse(msg.meta.to_string()));
  ASSERT_EQ(meta.request().service_name(), "example.EchoService");
  ASSERT_EQ(meta.compress_type(), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(meta.correlation_id(), 77);
  ASSERT_EQ(meta.attachment_size(), 3);
  ASSERT_EQ(msg.payload.to_string(), "zzzzzzATT");
}

TEST_CPU(protocol_compress_mappings) {
  // hulu_pbrpc_protocol.cc:58-98
  ASSERT_EQ(Hulu2CompressType(HULU_COMPRESS_TYPE_SNAPPY), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(Hulu2CompressType(HULU_COMPRESS_TYPE_ZLIB), COMPRESS_TYPE_ZLIB);
  ASSERT_EQ(Hulu2CompressType((HuluCompressType)9), COMPRESS_TYPE_NONE);
  ASSERT_EQ(CompressType2Hulu(COMPRESS_TYPE_SNAPPY), HULU_COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(CompressType2Hulu(COMPRESS_TYPE_LZ4), HULU_COMPRESS_TYPE_NONE);
  // sofa: snappy is 3 on the wire; LZ4 (4) has no mapping back
  ASSERT_EQ((int)CompressType2Sofa(COMPRESS_TYPE_SNAPPY), 3);
  ASSERT_EQ(Sofa2CompressType(SOFA_COMPRESS_TYPE_SNAPPY), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(Sofa2CompressType(SOFA_COMPRESS_TYPE_GZIP), COMPRESS_TYPE_GZIP);
  ASSERT_EQ(Sofa2CompressType(SOFA_COMPRESS_TYPE_LZ4), COMPRESS_TYPE_NONE);
  ASSERT_EQ(CompressType2Sofa(COMPRESS_TYPE_LZ4), SOFA_COMPRESS_TYPE_NONE);
  // nova: bit 0 of nshead.version
  ASSERT_EQ(NovaCompressTypeFromVersion(0x1), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(NovaCompressTypeFromVersion(0x3), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(NovaCompressTypeFromVersion(0x2), COMPRESS_TYPE_NONE);
  CompressType t = COMPRESS_TYPE_SNAPPY;
  ASSERT_EQ(NovaResponseVersion(&t), NOVA_SNAPPY_COMPRESS_FLAG);
  t = COMPRESS_TYPE_GZIP;
  ASSERT_EQ(NovaResponseVersion(&t), 0);
  ASSERT_EQ(t, COMPRESS_TYPE_NONE);
  // public_pbrpc: head compress_type 1 == snappy
  ASSERT_EQ(PublicPbrpc2CompressType(1), COMPRESS_TYPE_SNAPPY);
  ASSERT_EQ(PublicPbrpc2CompressType(0), COMPRESS_TYPE_NONE);
  ASSERT_EQ(PublicPbrpc2CompressType(3), COMPRESS_TYPE_NONE);
  // request-side support checks
  SnappyMessageProto req;
  req.set_text("x");
  Controller c1;
  c1.set_request_compress_type(COMPRESS_TYPE_GZIP);
  cord_buf b;
  SerializeNovaRequest(&b, &c1, &req);
  ASSERT_EQ(c1.ErrorCode(), EREQUEST);
  ASSERT_EQ(c1.ErrorText(), "nova_pbrpc protocol doesn't support compress_type=2");
  Controller c2;
  c2.set_request_compress_type(COMPRESS_TYPE_LZ4);
  SerializePublicPbrpcRequest(&b, &c2, &req);
  ASSERT_EQ(c2.ErrorText(), "public_pbrpc doesn't support compress type=4");
  Controller c3;  // NONE passes through to SerializeRequestDefault
  SerializePublicPbrpcRequest(&b, &c3, &req);
  ASSERT_FALSE(c3.Failed());
  ASSERT_EQ(b.to_string(), req.SerializeAsString());
}

// ---------------------------------------------------------------- GPU tests
TEST_GPU(nova_and_public_snappy_bodies) {
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  // nova: request compressed because the controller says SNAPPY; the server
  // reads the flag from nshead.version and parses through the handler
  SnappyMessageProto req, got;
  req.set_text(text(5000, 5));
  req.add_numbers(-1);
  Controller cc;
  cc.set_request_compress_type(COMPRESS_TYPE_SNAPPY);
  cord_buf body;
  SerializeNovaRequest(&body, &cc, &req);
  ASSERT_FALSE(cc.Failed());
  const uint16_t version = NOVA_SNAPPY_COMPRESS_FLAG;
  ASSERT_TRUE(ParseFromCompressedData(body, &got, NovaCompressTypeFromVersion(version)));
  ASSERT_EQ(got.SerializeAsString(), req.SerializeAsString());
  // public_pbrpc: the response string is compressed with the flat API
  // (public_pbrpc_protocol.cc:137-141) and parsed back by type 1 -> SNAPPY
  const std::string res = req.SerializeAsString();
  std::string tmp;
  flare::snappy::Compress(res.data(), res.size(), &tmp);
  cord_buf wire;
  wire.append(tmp);
  SnappyMessageProto got2;
  ASSERT_TRUE(ParseFromCompressedData(wire, &got2, PublicPbrpc2CompressType(PUBLIC_PBRPC_COMPRESS_TYPE)));
  ASSERT_EQ(got2.text(), req.text());
}

TEST_GPU(snappy_request_response_round_trip) {
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  for (size_t n : {0ul, 1ul, 200ul, 4093ul, 70000ul, 300000ul}) {
    SnappyMessageProto req, got_req, res, got_res;
    req.set_text(text(n, n + 1));
    for (int i = 0; i < 20; ++i) req.add_numbers(i * 1000 - 5000);
    Controller cc;
    cc.set_request_compress_type(COMPRESS_TYPE_SNAPPY);
    cc.request_attachment().append("att", 3);
    cord_buf body;
    SerializeRequestDefault(&body, &cc, &req);
    ASSERT_FALSE(cc.Failed());
    cord_buf wire;
    PackRpcRequest(&wire, 1, "S", "M", &cc, body);
    MostCommonMessage msg;
    ASSERT_EQ(ParseRpcMessage(&wire, &msg), PARSE_OK);
    Controller sc;
    RpcMeta meta;
    ASSERT_TRUE(ProcessRpcRequest(&msg, &sc, &got_req, &meta));
    ASSERT_FALSE(sc.Failed());
    ASSERT_EQ(meta.compress_type(), COMPRESS_TYPE_SNAPPY);
    ASSERT_EQ(got_req.SerializeAsString(), req.SerializeAsString());
    ASSERT_EQ(sc.request_attachment().to_string(), "att");

    sc.set_response_compress_type(COMPRESS_TYPE_SNAPPY);
    res.set_text(text(n / 2, n + 7));
    cord_buf out;
    SendRpcResponse(meta.correlation_id(), &sc, &res, &out);
    MostCommonMessage rmsg;
    ASSERT_EQ(ParseRpcMessage(&out, &rmsg), PARSE_OK);
    Controller cc2;
    ProcessRpcResponse(&rmsg, &cc2, &got_res);
    ASSERT_FALSE(cc2.Failed());
    ASSERT_EQ(cc2.response_compress_type(), COMPRESS_TYPE_SNAPPY);
    ASSERT_EQ(got_res.text(), res.text());
  }
}

TEST_GPU(corrupt_snappy_body_is_erequest) {
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  RpcMeta meta;
  meta.mutable_request()->set_service_name("S");
  meta.mutable_request()->set_method_name("M");
  meta.set_compress_type(COMPRESS_TYPE_SNAPPY);
  cord_buf wire = frame_of(meta, std::string("\x0a\x00\x61\x62", 4));  // says 10 bytes, has 2
  MostCommonMessage msg;
  ASSERT_EQ(ParseRpcMessage(&wire, &msg), PARSE_OK);
  Controller sc;
  SnappyMessageProto req;
  ASSERT_TRUE(ProcessRpcRequest(&msg, &sc, &req, nullptr));
  ASSERT_EQ(sc.ErrorCode(), EREQUEST);
  ASSERT_EQ(sc.ErrorText(), "Fail to parse request message, CompressType=snappy, request_size=4");
}

TEST_GPU(decode_frames_one_batch) {
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  // a receive buffer holding many pipelined frames: SNAPPY, NONE, a corrupt
  // one, one with an attachment, and a trailing partial frame
  cord_buf stream;
  std::vector<std::string> bodies;
  std::vector<bool> expect_ok;
  const int kFrames = 300;
  for (int i = 0; i < kFrames; ++i) {
    std::string b = text((size_t)(i * 131) % 20000, i);
    RpcMeta meta;
    meta.mutable_request()->set_service_name("S");
    meta.mutable_request()->set_method_name("M");
    meta.set_correlation_id(i);
    cord_buf payload;
    bool ok = true;
    if (i % 7 == 3) {
      meta.set_compress_type(COMPRESS_TYPE_NONE);
      payload.append(b);
    } else if (i % 50 == 11) {
      meta.set_compress_type(COMPRESS_TYPE_SNAPPY);
      payload.append("\x05\x00\x61", 3);  // truncated literal
      ok = false;
    } else {
      meta.set_compress_type(COMPRESS_TYPE_SNAPPY);
      cord_buf raw;
      raw.append(b);
      ASSERT_TRUE(SnappyCompress(raw, &payload));
    }
    if (i % 5 == 0) {
      meta.set_attachment_size(4);
      payload.append("ATT!", 4);
    }
    SerializeRpcHeaderAndMeta(&stream, meta, payload.size());
    stream.append(payload);
    bodies.push_back(b);
    expect_ok.push_back(ok);
  }
  stream.append("PRPC\0\0", 6);
  std::vector<DecodedFrame> frames;
  ParseError stop = PARSE_OK;
  ASSERT_EQ(DecodeRpcFrames(&stream, &frames, &stop), (size_t)kFrames);
  ASSERT_EQ(stop, PARSE_ERROR_NOT_ENOUGH_DATA);
  ASSERT_EQ(stream.size(), 6u);
  for (int i = 0; i < kFrames; ++i) {
    ASSERT_EQ(frames[i].ok, (bool)expect_ok[i]);
    ASSERT_EQ(frames[i].meta.correlation_id(), i);
    if (expect_ok[i]) ASSERT_EQ(frames[i].body.to_string(), bodies[i]);
    ASSERT_EQ(frames[i].attachment.to_string(), i % 5 == 0 ? "ATT!" : "");
  }
}

TEST_GPU(dump_then_batch_decompress) {
  ASSERT_EQ(GlobalInitializeSnappyGpu(), 0);
  const std::string dir = tmpdir("gpu");
  std::vector<std::string> bodies;
  {
    RpcDumpWriter w(dir, 50, 8);
    for (int i = 0; i < 120; ++i) {
      SampledRequest s;
      s.meta.set_service_name("svc");
      s.meta.set_method_name("m");
      s.meta.set_protocol_type(PROTOCOL_BAIDU_STD);
      const std::string b = text(1000 + 613 * i, 3 * i);
      cord_buf raw;
      raw.append(b);
      if (i % 4 == 0) {
        s.meta.set_compress_type(COMPRESS_TYPE_NONE);
        s.request.append(b);
      } else {
        s.meta.set_compress_type(COMPRESS_TYPE_SNAPPY);
        ASSERT_TRUE(SnappyCompress(raw, &s.request));
      }
      s.meta.set_attachment_size(2);
      s.request.append("at", 2);
      bodies.push_back(b);
      ASSERT_TRUE(w.Dump(s));
    }
  }
  std::vector<std::unique_ptr<SampledRequest>> owned;
  SampleIterator it(dir);
  while (auto s = it.Next()) owned.push_back(std::move(s));
  ASSERT_EQ(owned.size(), bodies.size());
  std::vector<const SampledRequest*> ptrs;
  for (auto& s : owned) ptrs.push_back(s.get());
  std::vector<cord_buf> out;
  std::vector<bool> ok;
  ASSERT_EQ(DecompressSamples(ptrs, &out, &ok), bodies.size());
  for (size_t i = 0; i < bodies.size(); ++i) ASSERT_EQ(out[i].to_string(), bodies[i]);
}

// ------------------------------------------------------------------- driver
static int emit(const char* dir) {
  mkdir(dir, 0755);
  const auto mc = meta_cases();
  for (size_t i = 0; i < mc.size(); ++i) {
    std::ofstream f(std::string(dir) + "/meta_" + std::to_string(i) + ".bin", std::ios::binary);
    f << mc[i].SerializeAsString();
  }
  const auto dc = dump_meta_cases();
  for (size_t i = 0; i < dc.size(); ++i) {
    std::ofstream f(std::string(dir) + "/dump_meta_" + std::to_string(i) + ".bin", std::ios::binary);
    f << dc[i].SerializeAsString();
  }
  // one full request frame (header + meta + payload + attachment)
  Controller cc;
  cc.set_request_compress_type(COMPRESS_TYPE_NONE);
  cc.request_attachment().append("ATT", 3);
  cord_buf body, wire;
  body.append("payload-bytes", 13);
  PackRpcRequest(&wire, 5, "example.EchoService", "Echo", &cc, body);
  std::ofstream f(std::string(dir) + "/request_frame.bin", std::ios::binary);
  f << wire.to_string();
  printf("%zu %zu\n", mc.size(), dc.size());
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "--emit")) return emit(argv[2]);
  if (argc >= 3 && !strcmp(argv[1], "--parse-meta")) {
    RpcMeta m;
    if (!m.Parse(read_file(argv[2]))) {
      printf("PARSE_FAIL\n");
      return 0;
    }
    printf("%s\n", to_json(m).c_str());
    return 0;
  }
  if (argc >= 3 && !strcmp(argv[1], "--parse-dump-meta")) {
    RpcDumpMeta m;
    if (!m.Parse(read_file(argv[2]))) {
      printf("PARSE_FAIL\n");
      return 0;
    }
    printf("%s\n", to_json(m).c_str());
    return 0;
  }
  const bool want_gpu = argc > 1 && !strcmp(argv[1], "--gpu");
  int failures = 0, run = 0;
  for (auto& t : registry()) {
    if (t.gpu != want_gpu) continue;
    ++run;
    try {
      t.fn();
      printf("[ OK ] %s\n", t.name);
    } catch (Failure&) {
      ++failures;
      printf("[FAIL] %s\n", t.name);
    }
  }
  printf("%d tests, %d failures\n", run, failures);
  return failures ? 1 : 0;
}

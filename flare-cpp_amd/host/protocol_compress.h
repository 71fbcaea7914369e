// protocol_compress.h -- how the other RPC protocols name the snappy codec
// on the wire: every mapping that routes a body to
// the COMPRESS_TYPE_SNAPPY handler, restated with the reference's values and
// its fallbacks for types a protocol cannot carry.
//
//   hulu_pbrpc   /root/reference/flare/rpc/policy/hulu_pbrpc_protocol.cc:58-98
//   sofa_pbrpc   sofa_pbrpc_meta.proto:25-31, sofa_pbrpc_protocol.cc:52-87
//   nova_pbrpc   nova_pbrpc_protocol.cc:50, :68-70, :94-101, :141-142,
//                :156-163, :187-190 (snappy = bit 0 of nshead.version)
//   public_pbrpc public_pbrpc_protocol.cc:57, :87-88, :137-141, :191-192,
//                :218-222, :251-252 (compress_type == 1 means snappy; the
//                response is compressed with the flat snappy::Compress, which
//                this build's host/snappy.h provides on the GPU)
#pragma once

#include <cstdint>

#include "baidu_rpc_protocol.h"
#include "compress.h"

namespace flare::rpc::policy {

// ---- hulu_pbrpc
enum HuluCompressType {
  HULU_COMPRESS_TYPE_NONE = 0,
  HULU_COMPRESS_TYPE_SNAPPY = 1,
  HULU_COMPRESS_TYPE_GZIP = 2,
  HULU_COMPRESS_TYPE_ZLIB = 3,
};
// Unknown values map to NONE (logged), as :75-77.
CompressType Hulu2CompressType(HuluCompressType type);
// LZ4 and unknown types map to NONE (logged), as :90-96.
HuluCompressType CompressType2Hulu(CompressType type);

// ---- sofa_pbrpc
enum SofaCompressType {
  SOFA_COMPRESS_TYPE_NONE = 0,
  SOFA_COMPRESS_TYPE_GZIP = 1,
  SOFA_COMPRESS_TYPE_ZLIB = 2,
  SOFA_COMPRESS_TYPE_SNAPPY = 3,
  SOFA_COMPRESS_TYPE_LZ4 = 4,
};
// SOFA_COMPRESS_TYPE_LZ4 has no case in the reference and falls to the
// default: NONE (logged), as :62-64.
CompressType Sofa2CompressType(SofaCompressType type);
// LZ4 and unknown types map to NONE (logged), as :78-84.
SofaCompressType CompressType2Sofa(CompressType type);

// ---- nova_pbrpc: snappy is bit 0 of nshead.version
constexpr uint16_t NOVA_SNAPPY_COMPRESS_FLAG = 0x1;
CompressType NovaCompressTypeFromVersion(uint16_t nshead_version);
// Server side (:94-101): SNAPPY sets the flag; any other non-NONE type is
// logged and the response goes out uncompressed (*type becomes NONE).
uint16_t NovaResponseVersion(CompressType* type);
// Client side (SerializeNovaRequest :156-163): NONE or SNAPPY only, else
// EREQUEST on the controller; then SerializeRequestDefault.
void SerializeNovaRequest(cord_buf* buf, Controller* cntl, const Message* request);

// ---- public_pbrpc: compress_type 1 in the head means snappy
constexpr uint32_t PUBLIC_PBRPC_COMPRESS_TYPE = 1;
CompressType PublicPbrpc2CompressType(uint32_t head_compress_type);
// Client side (SerializePublicPbrpcRequest :218-222): NONE or SNAPPY only.
void SerializePublicPbrpcRequest(cord_buf* buf, Controller* cntl, const Message* request);

}  // namespace flare::rpc::policy

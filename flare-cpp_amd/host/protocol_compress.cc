// protocol_compress.cc -- see protocol_compress.h.
#include "protocol_compress.h"

#include <cstdio>

namespace flare::rpc::policy {

CompressType Hulu2CompressType(HuluCompressType type) {
  switch (type) {
    case HULU_COMPRESS_TYPE_NONE: return COMPRESS_TYPE_NONE;
    case HULU_COMPRESS_TYPE_SNAPPY: return COMPRESS_TYPE_SNAPPY;
    case HULU_COMPRESS_TYPE_GZIP: return COMPRESS_TYPE_GZIP;
    case HULU_COMPRESS_TYPE_ZLIB: return COMPRESS_TYPE_ZLIB;
  }
  fprintf(stderr, "[ERROR] Unknown HuluCompressType=%d\n", (int)type);
  return COMPRESS_TYPE_NONE;
}

HuluCompressType CompressType2Hulu(CompressType type) {
  switch (type) {
    case COMPRESS_TYPE_NONE: return HULU_COMPRESS_TYPE_NONE;
    case COMPRESS_TYPE_SNAPPY: return HULU_COMPRESS_TYPE_SNAPPY;
    case COMPRESS_TYPE_GZIP: return HULU_COMPRESS_TYPE_GZIP;
    case COMPRESS_TYPE_ZLIB: return HULU_COMPRESS_TYPE_ZLIB;
    case COMPRESS_TYPE_LZ4:
      fprintf(stderr, "[ERROR] Hulu doesn't support LZ4\n");
      return HULU_COMPRESS_TYPE_NONE;
  }
  fprintf(stderr, "[ERROR] Unknown CompressType=%d\n", (int)type);
  return HULU_COMPRESS_TYPE_NONE;
}

CompressType Sofa2CompressType(SofaCompressType type) {
  switch (type) {
    case SOFA_COMPRESS_TYPE_NONE: return COMPRESS_TYPE_NONE;
    case SOFA_COMPRESS_TYPE_SNAPPY: return COMPRESS_TYPE_SNAPPY;
    case SOFA_COMPRESS_TYPE_GZIP: return COMPRESS_TYPE_GZIP;
    case SOFA_COMPRESS_TYPE_ZLIB: return COMPRESS_TYPE_ZLIB;
    default: break;  // SOFA_COMPRESS_TYPE_LZ4 included
  }
  fprintf(stderr, "[ERROR] Unknown SofaCompressType=%d\n", (int)type);
  return COMPRESS_TYPE_NONE;
}

SofaCompressType CompressType2Sofa(CompressType type) {
  switch (type) {
    case COMPRESS_TYPE_NONE: return SOFA_COMPRESS_TYPE_NONE;
    case COMPRESS_TYPE_SNAPPY: return SOFA_COMPRESS_TYPE_SNAPPY;
    case COMPRESS_TYPE_GZIP: return SOFA_COMPRESS_TYPE_GZIP;
    case COMPRESS_TYPE_ZLIB: return SOFA_COMPRESS_TYPE_ZLIB;
    case COMPRESS_TYPE_LZ4:
      fprintf(stderr, "[ERROR] sofa-pbrpc does not support LZ4\n");
      return SOFA_COMPRESS_TYPE_NONE;
  }
  fprintf(stderr, "[ERROR] Unknown SofaCompressType=%d\n", (int)type);
  return SOFA_COMPRESS_TYPE_NONE;
}

CompressType NovaCompressTypeFromVersion(uint16_t nshead_version) {
  return (nshead_version & NOVA_SNAPPY_COMPRESS_FLAG) ? COMPRESS_TYPE_SNAPPY : COMPRESS_TYPE_NONE;
}

uint16_t NovaResponseVersion(CompressType* type) {
  if (*type == COMPRESS_TYPE_SNAPPY) return NOVA_SNAPPY_COMPRESS_FLAG;
  if (*type != COMPRESS_TYPE_NONE) {
    fprintf(stderr, "[WARNING] nova_pbrpc protocol doesn't support compress_type=%d\n", (int)*type);
    *type = COMPRESS_TYPE_NONE;
  }
  return 0;
}

void SerializeNovaRequest(cord_buf* buf, Controller* cntl, const Message* request) {
  const CompressType type = cntl->request_compress_type();
  if (type != COMPRESS_TYPE_NONE && type != COMPRESS_TYPE_SNAPPY)
    return cntl->SetFailed(EREQUEST, "nova_pbrpc protocol doesn't support compress_type=%d", (int)type);
  SerializeRequestDefault(buf, cntl, request);
}

CompressType PublicPbrpc2CompressType(uint32_t head_compress_type) {
  return head_compress_type == PUBLIC_PBRPC_COMPRESS_TYPE ? COMPRESS_TYPE_SNAPPY : COMPRESS_TYPE_NONE;
}

void SerializePublicPbrpcRequest(cord_buf* buf, Controller* cntl, const Message* request) {
  const CompressType type = cntl->request_compress_type();
  if (type != COMPRESS_TYPE_NONE && type != COMPRESS_TYPE_SNAPPY)
    return cntl->SetFailed(EREQUEST, "public_pbrpc doesn't support compress type=%d", (int)type);
  SerializeRequestDefault(buf, cntl, request);
}

}  // namespace flare::rpc::policy

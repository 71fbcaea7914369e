// snappy.h -- GPU-backed flat Snappy API with the reference's names and
// semantics (/root/reference/flare/io/snappy/snappy.h:62-190).  Covers the
// second call site of the hot path, public_pbrpc's direct
// flare::snappy::Compress(const char*, size_t, std::string*)
// (/root/reference/flare/rpc/policy/public_pbrpc_protocol.cc:137-142).
// Large calls are (batched) GPU jobs, small ones run the host codec; bytes
// and verdicts are identical to the reference.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "cord_buf.h"

struct iovec;

namespace flare::snappy {

// snappy.cc:55-77
size_t MaxCompressedLength(size_t source_bytes);

// snappy.cc:1313-1322.  Returns the compressed length.
size_t Compress(const char* input, size_t input_length, std::string* output);

// snappy.cc:1239-1251: strict header (Parse32WithLimit), then decode.
bool Uncompress(const char* compressed, size_t compressed_length, std::string* uncompressed);

// snappy.cc:1301-1311.  `compressed` must hold MaxCompressedLength(n) bytes.
void RawCompress(const char* input, size_t input_length, char* compressed,
                 size_t* compressed_length);

// snappy.cc:1229-1237 (lenient header, like the Source path).  `uncompressed`
// must hold the header's length (GetUncompressedLength).
bool RawUncompress(const char* compressed, size_t compressed_length, char* uncompressed);

// snappy.cc:235-244 (strict header).
bool GetUncompressedLength(const char* compressed, size_t compressed_length, size_t* result);

// snappy.cc:1290-1294 (the device's validate-only pass for large inputs).
bool IsValidCompressedBuffer(const char* compressed, size_t compressed_length);

// snappy.h:152-164, snappy.cc:1124-1139 (SnappyIOVecWriter): decodes into
// the iovecs in order; false if the stream is invalid or the iovecs hold
// fewer bytes than the header length (what they hold then is unspecified).
bool RawUncompressToIOVec(const char* compressed, size_t compressed_length, const struct iovec* iov,
                          size_t iov_cnt);

// snappy.h:181-190, snappy.cc:1530-1535: appends what the reference's
// scattered writer would have produced before the first failing tag, and
// returns the reference's result (see snappy_cpu.h for its one quirk).
// Source fragments = the cord_buf's backing blocks.
size_t UncompressAsMuchAsPossible(const cord_buf& compressed, cord_buf* uncompressed);

}  // namespace flare::snappy

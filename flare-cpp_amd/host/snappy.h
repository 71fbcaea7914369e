// snappy.h -- GPU-backed flat Snappy API with the reference's names and
// semantics (/root/reference/flare/io/snappy/snappy.h:62-190).  Covers the
// second call site of the hot path, public_pbrpc's direct
// flare::snappy::Compress(const char*, size_t, std::string*)
// (/root/reference/flare/rpc/policy/public_pbrpc_protocol.cc:137-142).
// Every call is one (batched) GPU job; bytes are identical to the reference.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

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

// snappy.cc:1290-1294.
bool IsValidCompressedBuffer(const char* compressed, size_t compressed_length);

}  // namespace flare::snappy

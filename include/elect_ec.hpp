// elect_ec.hpp — header-only C++17 mirror of ELECT's Java coder API
// (org.apache.cassandra.io.erasurecode) over the C ABI in elect_ec.h.
//
// Same class names, argument meaning, checks and exceptions as the Java
// (JEC/ = src/elect/src/java/org/apache/cassandra/io/erasurecode):
//   ErasureCoderOptions      JEC/ErasureCoderOptions.java
//   ErasureEncoder::encode   JEC/ErasureEncoder.java:38-47
//   ErasureEncoder::encodeUpdate  JEC/ErasureEncoder.java:58-71
//   ErasureDecoder::decode   JEC/ErasureDecoder.java:30-39
//   NativeRSEncoder/Decoder  JEC/NativeRSEncoder.java, JEC/NativeRSDecoder.java
//   CoderUtil checks         JEC/CoderUtil.java:49-107
//   state validation         JEC/ByteBufferEncodingState.java, JEC/ByteBufferDecodingState.java
// A ByteBuffer is a (pointer, position, limit, direct) view; like the JNI glue
// (EC/jni_common.c:62-108) the native call receives base + position.
#pragma once

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "elect_ec.h"

namespace elect {
namespace erasurecode {

struct ErasureCodeException : std::runtime_error {  // org.apache.cassandra.exceptions.ErasureCodeException
    using std::runtime_error::runtime_error;
};
struct IOException : std::runtime_error {  // java.io.IOException
    using std::runtime_error::runtime_error;
};
struct InternalError : std::runtime_error {  // java.lang.InternalError (EC/jni_common.c:72, 96)
    using std::runtime_error::runtime_error;
};
struct NullPointerException : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct DeviceError : std::runtime_error {  // engine status codes (include/elect_ec.h)
    int status;
    DeviceError(int st, const std::string& what) : std::runtime_error(what + ": " + elect_ec_strerror(st)), status(st) {}
};

// java.nio.ByteBuffer, the subset the coder path reads.  Not owning.
struct ByteBuffer {
    unsigned char* base = nullptr;
    size_t pos = 0;
    size_t lim = 0;
    bool direct = true;

    static ByteBuffer wrapDirect(unsigned char* p, size_t n) { return ByteBuffer{p, 0, n, true}; }
    size_t position() const { return pos; }
    size_t remaining() const { return lim - pos; }
    bool isDirect() const { return direct; }
    unsigned char* address() const { return base + pos; }  // GetDirectBufferAddress + position
};

using Buffers = std::vector<ByteBuffer*>;  // nullptr = Java null

class ErasureCoderOptions {
public:
    ErasureCoderOptions(int numDataUnits, int numParityUnits, bool allowVerboseDump = false)
        : k_(numDataUnits), m_(numParityUnits), verbose_(allowVerboseDump) {}
    int getNumDataUnits() const { return k_; }
    int getNumParityUnits() const { return m_; }
    int getNumAllUnits() const { return k_ + m_; }
    bool allowVerboseDump() const { return verbose_; }

private:
    int k_, m_;
    bool verbose_;
};

namespace detail {
inline ByteBuffer* firstValid(const Buffers& b)
{
    for (auto* x : b)
        if (x) return x;
    throw ErasureCodeException("Invalid inputs, all being null!");
}

inline void checkBuffers(const Buffers& b, size_t len, bool direct)  // JEC/CoderUtil.java:93-107
{
    for (auto* x : b) {
        if (!x) throw ErasureCodeException("Invalid buffer, being null");
        if (x->remaining() != len) throw ErasureCodeException("Invalid buffer, not of length " + std::to_string(len));
        if (x->isDirect() != direct)
            throw ErasureCodeException(std::string("Invalid buffer, isDirect should be ") + (direct ? "true" : "false"));
    }
}

inline void check(int st, const char* what)
{
    if (st < 0) {
        if (st == ELECT_EC_EINVAL) throw ErasureCodeException(std::string(what) + ": " + elect_ec_strerror(st));
        throw DeviceError(st, what);
    }
}
}  // namespace detail

class ErasureCoder {
public:
    explicit ErasureCoder(const ErasureCoderOptions& o) : options_(o) {}
    virtual ~ErasureCoder() = default;
    int getNumDataUnits() const { return options_.getNumDataUnits(); }
    int getNumParityUnits() const { return options_.getNumParityUnits(); }
    int getNumAllUnits() const { return options_.getNumAllUnits(); }
    const ErasureCoderOptions& getOptions() const { return options_; }
    bool allowVerboseDump() const { return options_.allowVerboseDump(); }
    virtual void release() {}

private:
    ErasureCoderOptions options_;
};

class ErasureEncoder : public ErasureCoder {
public:
    using ErasureCoder::ErasureCoder;

    void encode(const Buffers& inputs, const Buffers& outputs)  // JEC/ErasureEncoder.java:38
    {
        const size_t len = validate(inputs, outputs);
        if (len == 0) return;
        doEncode(inputs, outputs, len);
    }

    void encodeUpdate(const Buffers& targetCodingBlock, const Buffers& parityBuffers, int targetDataIndex)
    {
        const size_t len = validate(targetCodingBlock, parityBuffers);
        if (len == 0) return;
        doEncodeUpdate(targetCodingBlock, parityBuffers, targetDataIndex, len);
    }

protected:
    virtual void doEncode(const Buffers& in, const Buffers& out, size_t len) = 0;
    virtual void doEncodeUpdate(const Buffers& in, const Buffers& out, int target, size_t len) = 0;

private:
    size_t validate(const Buffers& inputs, const Buffers& outputs)  // JEC/ByteBufferEncodingState.java:34-55
    {
        ByteBuffer* v = detail::firstValid(inputs);
        const size_t len = v->remaining();
        const bool direct = v->isDirect();
        const int k = getNumDataUnits(), m = getNumParityUnits();
        if (static_cast<int>(inputs.size()) != k && static_cast<int>(inputs.size()) != m + 2)
            throw ErasureCodeException("Invalid inputs length for encoding!");
        if (static_cast<int>(outputs.size()) != m) throw ErasureCodeException("Invalid outputs length for encoding!");
        detail::checkBuffers(inputs, len, direct);
        detail::checkBuffers(outputs, len, direct);
        return len;
    }
};

class ErasureDecoder : public ErasureCoder {
public:
    using ErasureCoder::ErasureCoder;

    void decode(const Buffers& inputs, const std::vector<int>& decodeIndexes, const std::vector<int>& erasedIndexes,
                const Buffers& outputs)  // JEC/ErasureDecoder.java:30
    {
        ByteBuffer* v = detail::firstValid(inputs);
        const size_t len = v->remaining();
        const bool direct = v->isDirect();
        for (auto* o : outputs)
            if (!o) throw NullPointerException("outputs[i].position()");  // JEC/ByteBufferDecodingState.java:58
        const int k = getNumDataUnits(), m = getNumParityUnits();
        if (static_cast<int>(inputs.size()) < k) throw ErasureCodeException("Invalid inputs length for decoding");
        if (erasedIndexes.size() != outputs.size())
            throw ErasureCodeException("erasedIndexes and outputs mismatch in length");
        if (static_cast<int>(erasedIndexes.size()) > m) throw ErasureCodeException("Too many erased, not recoverable");
        int valid = 0;
        for (auto* b : inputs) {
            if (!b) continue;
            if (b->remaining() != len) throw ErasureCodeException("Invalid buffer, not of length " + std::to_string(len));
            if (b->isDirect() != direct) throw ErasureCodeException("Invalid buffer, isDirect mismatch");
            ++valid;
        }
        if (valid < k) throw ErasureCodeException("No enough valid inputs are provided, not recoverable");
        for (auto* b : outputs) {
            if (b->remaining() != len) throw ErasureCodeException("Invalid buffer, not of length " + std::to_string(len));
            if (b->isDirect() != direct) throw ErasureCodeException("Invalid buffer, isDirect mismatch");
        }
        if (len == 0) return;
        doDecode(inputs, decodeIndexes, erasedIndexes, outputs, len);
    }

protected:
    virtual void doDecode(const Buffers& in, const std::vector<int>& dec, const std::vector<int>& era,
                          const Buffers& out, size_t len) = 0;
};

namespace detail {
// getInputs / getOutputs (EC/jni_common.c:62-108): count check, then addresses.
inline std::vector<unsigned char*> addresses(const Buffers& b, size_t expected, const char* what)
{
    if (b.size() != expected) throw InternalError(what);
    std::vector<unsigned char*> p;
    p.reserve(b.size());
    for (auto* x : b) {
        if (!x) throw InternalError(what);
        p.push_back(x->address());
    }
    return p;
}
}  // namespace detail

class NativeRSEncoder : public ErasureEncoder {
public:
    explicit NativeRSEncoder(const ErasureCoderOptions& o) : ErasureEncoder(o)
    {
        std::unique_lock<std::shared_mutex> w(lock_);
        detail::check(elect_ec_coder_create(o.getNumDataUnits(), o.getNumParityUnits(), &coder_), "initImpl");
    }
    ~NativeRSEncoder() override { release(); }

    void release() override
    {
        std::unique_lock<std::shared_mutex> w(lock_);
        elect_ec_coder_destroy(coder_);
        coder_ = nullptr;
    }

protected:
    void doEncode(const Buffers& in, const Buffers& out, size_t len) override
    {
        std::shared_lock<std::shared_mutex> r(lock_);
        if (!coder_) throw IOException("NativeRSEncoder closed");
        auto i = detail::addresses(in, getNumDataUnits(), "Invalid inputs");
        auto o = detail::addresses(out, getNumParityUnits(), "Invalid outputs");
        detail::check(elect_ec_encode(coder_, i.data(), o.data(), len), "encode");
    }

    void doEncodeUpdate(const Buffers& in, const Buffers& out, int target, size_t len) override
    {
        std::shared_lock<std::shared_mutex> r(lock_);
        if (!coder_) throw IOException("NativeRSEncoder closed");
        auto i = detail::addresses(in, 2 + getNumParityUnits(), "Invalid inputs");
        auto o = detail::addresses(out, getNumParityUnits(), "Invalid outputs");
        detail::check(elect_ec_encode_update(coder_, i.data(), target, o.data(), len), "encodeUpdate");
    }

private:
    std::shared_mutex lock_;  // JEC/NativeRSEncoder.java:33 (ReentrantReadWriteLock)
    elect_ec_coder* coder_ = nullptr;
};

class NativeRSDecoder : public ErasureDecoder {
public:
    explicit NativeRSDecoder(const ErasureCoderOptions& o, int mode = ELECT_EC_DECODE_COMPAT)
        : ErasureDecoder(o), mode_(mode)
    {
        std::unique_lock<std::shared_mutex> w(lock_);
        detail::check(elect_ec_coder_create(o.getNumDataUnits(), o.getNumParityUnits(), &coder_), "initImpl");
    }
    ~NativeRSDecoder() override { release(); }

    void release() override
    {
        std::unique_lock<std::shared_mutex> w(lock_);
        elect_ec_coder_destroy(coder_);
        coder_ = nullptr;
    }

    int lastStatus() const { return last_; }

protected:
    void doDecode(const Buffers& in, const std::vector<int>& dec, const std::vector<int>& era, const Buffers& out,
                  size_t len) override
    {
        std::shared_lock<std::shared_mutex> r(lock_);
        if (!coder_) throw IOException("NativeRSDecoder closed");
        const int k = getNumDataUnits();
        if (static_cast<int>(dec.size()) < k) throw InternalError("Invalid decodeIndexes");
        auto i = detail::addresses(in, k, "Invalid inputs");
        auto o = detail::addresses(out, era.size(), "Invalid outputs");
        last_ = elect_ec_decode(coder_, i.data(), dec.data(), era.data(), static_cast<int>(era.size()), o.data(), len,
                                mode_);
        detail::check(last_, "decode");
    }

private:
    std::shared_mutex lock_;
    elect_ec_coder* coder_ = nullptr;
    int mode_;
    int last_ = ELECT_EC_OK;
};

}  // namespace erasurecode

// ---------------------------------------------------------------------------
// Checked device-batch calls for C++ callers (the elect_ec_*_batch entry points
// of elect_ec.h).  The C ABI addresses a device batch from its base and strides
// alone, so a descriptor with fewer stripes, units or bytes than the call
// implies is read or written out of bounds on the device.  A DeviceBatch states
// its geometry (and, optionally, the bytes allocated from base), and every call
// below checks it before anything is enqueued: the same checks as the Python
// wrappers (elect_amd/batch.py).  std::invalid_argument on a mismatch.
// ---------------------------------------------------------------------------
namespace device {

// `stripes` stripes of `units` units of `len` bytes: unit i of stripe s at
// base + s*stripe_stride + i*unit_stride.  `bytes` = the allocation behind base
// (0 = unknown: geometry checks only).
struct DeviceBatch {
    void* base = nullptr;
    size_t stripes = 0;
    size_t units = 0;
    size_t len = 0;
    size_t stripe_stride = 0;
    size_t unit_stride = 0;
    size_t bytes = 0;

    // a contiguous [stripes][units][len] block
    static DeviceBatch contiguous(void* p, size_t stripes, size_t units, size_t len)
    {
        return DeviceBatch{p, stripes, units, len, units * len, len, stripes * units * len};
    }
    // units [first, first + n) of this batch (same stripes and strides)
    DeviceBatch slice(size_t first, size_t n) const
    {
        if (first + n > units) throw std::invalid_argument("DeviceBatch::slice past the last unit");
        DeviceBatch b = *this;
        b.base = static_cast<unsigned char*>(base) + first * unit_stride;
        b.units = n;
        if (bytes) b.bytes = bytes - first * unit_stride;
        return b;
    }
    elect_ec_shards shards() const { return elect_ec_shards{base, stripe_stride, unit_stride}; }
};

namespace detail {
inline void check_batch(const char* name, const DeviceBatch& b, size_t stripes, size_t len, size_t need)
{
    auto fail = [&](const std::string& why) {
        throw std::invalid_argument(std::string(name) + ": " + why + " (expected [" + std::to_string(stripes) + ", >=" +
                                    std::to_string(need) + ", " + std::to_string(len) + "], got [" +
                                    std::to_string(b.stripes) + ", " + std::to_string(b.units) + ", " +
                                    std::to_string(b.len) + "])");
    };
    if (b.stripes != stripes || b.len != len || b.units < need) fail("shape mismatch");
    if (stripes && len && !b.base) fail("null base");
    if (b.bytes && stripes && need) {  // the farthest byte the call touches lies inside the allocation
        const size_t last = (stripes - 1) * b.stripe_stride + (need - 1) * b.unit_stride + len;
        if (last > b.bytes) fail("strides reach " + std::to_string(last) + " B past a " + std::to_string(b.bytes) + " B buffer");
    }
}

inline int max_index(const int* idx, int n)
{
    int m = -1;
    for (int i = 0; i < n; ++i) m = idx[i] > m ? idx[i] : m;
    return m;
}
}  // namespace detail

// elect_ec_encode_batch: data [B, >=k, L], parity [B, >=m, L].
inline int encode_batch(const elect_ec_coder* c, const DeviceBatch& data, const DeviceBatch& parity, void* stream)
{
    const size_t k = elect_ec_coder_num_data_units(c), m = elect_ec_coder_num_parity_units(c);
    detail::check_batch("data", data, data.stripes, data.len, k);
    detail::check_batch("parity", parity, data.stripes, data.len, m);
    return elect_ec_encode_batch(c, data.len, data.stripes, data.shards(), parity.shards(), stream);
}

// elect_ec_encode_batch_ex (content lengths and hashes: DEVICE arrays of
// [B][k] / [B][m] entries the caller sized; the C ABI reads them by index).
inline int encode_batch_ex(const elect_ec_coder* c, const DeviceBatch& data, const uint32_t* d_lengths,
                           const DeviceBatch& parity, int32_t* d_hashes, void* stream)
{
    const size_t k = elect_ec_coder_num_data_units(c), m = elect_ec_coder_num_parity_units(c);
    detail::check_batch("data", data, data.stripes, data.len, k);
    detail::check_batch("parity", parity, data.stripes, data.len, m);
    return elect_ec_encode_batch_ex(c, data.len, data.stripes, data.shards(), d_lengths, parity.shards(), d_hashes,
                                    stream);
}

// elect_ec_decode_batch: inputs [B, k (or max(decode_indexes)+1 with
// ELECT_EC_INPUTS_BY_UNIT), L], outputs [B, num_erased (or max(erased)+1 with
// ELECT_EC_OUTPUTS_BY_UNIT), L].
inline int decode_batch(const elect_ec_coder* c, const DeviceBatch& inputs, const int* decode_indexes,
                        const int* erased, int num_erased, const DeviceBatch& outputs, unsigned flags, int mode,
                        void* stream)
{
    const int k = elect_ec_coder_num_data_units(c);
    if (num_erased < 0 || (num_erased > 0 && !erased) || !decode_indexes)
        throw std::invalid_argument("decode_batch: bad index arrays");
    const size_t in_need = (flags & ELECT_EC_INPUTS_BY_UNIT) ? detail::max_index(decode_indexes, k) + 1 : k;
    const size_t out_need = (flags & ELECT_EC_OUTPUTS_BY_UNIT) ? detail::max_index(erased, num_erased) + 1
                                                               : static_cast<size_t>(num_erased);
    detail::check_batch("inputs", inputs, inputs.stripes, inputs.len, in_need);
    detail::check_batch("outputs", outputs, inputs.stripes, inputs.len, out_need);
    return elect_ec_decode_batch(c, inputs.len, inputs.stripes, inputs.shards(), decode_indexes, erased, num_erased,
                                 outputs.shards(), flags, mode, stream);
}

// elect_ec_encode_update_batch: old / new [B, >=1, L] (unit 0 used), parity
// in / out [B, >=m, L].
inline int encode_update_batch(const elect_ec_coder* c, int target, const DeviceBatch& old_data,
                               const DeviceBatch& new_data, const DeviceBatch& parity_in,
                               const DeviceBatch& parity_out, void* stream)
{
    const size_t m = elect_ec_coder_num_parity_units(c);
    detail::check_batch("old", old_data, old_data.stripes, old_data.len, 1);
    detail::check_batch("new", new_data, old_data.stripes, old_data.len, 1);
    detail::check_batch("parity_in", parity_in, old_data.stripes, old_data.len, m);
    detail::check_batch("parity_out", parity_out, old_data.stripes, old_data.len, m);
    return elect_ec_encode_update_batch(c, old_data.len, old_data.stripes, target,
                                        elect_ec_column{old_data.base, old_data.stripe_stride},
                                        elect_ec_column{new_data.base, new_data.stripe_stride}, parity_in.shards(),
                                        parity_out.shards(), stream);
}

}  // namespace device
}  // namespace elect

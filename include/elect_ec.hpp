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
}  // namespace elect

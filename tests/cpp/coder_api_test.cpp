// C++ driver for include/elect_ec.hpp (the Java coder API mirror).
//   coder_api_test cpu            error behaviour, no device needed (exit 0 = pass)
//   coder_api_test gpu OUTDIR     ErasureCodeTest.java:31-173 at codeLength 4099;
//                                 writes the buffers to OUTDIR for the Python side
//                                 to compare with tests/golden/erasure_code_test.json
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "elect_ec.hpp"

using namespace elect::erasurecode;

static int failures = 0;
#define EXPECT(cond)                                                     \
    do {                                                                 \
        if (!(cond)) {                                                   \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                  \
        }                                                                \
    } while (0)

template <class E, class F>
static bool throws(F&& f, const char* needle = nullptr)
{
    try {
        f();
    } catch (const E& e) {
        return !needle || std::strstr(e.what(), needle) != nullptr;
    } catch (...) {
        return false;
    }
    return false;
}

// java.util.Random(seed).nextBytes (JDK-specified 48-bit LCG)
struct JavaRandom {
    uint64_t seed;
    explicit JavaRandom(int64_t s) : seed((static_cast<uint64_t>(s) ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
    int32_t next32()
    {
        seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return static_cast<int32_t>(seed >> 16);
    }
    void nextBytes(std::vector<unsigned char>& b)
    {
        for (size_t i = 0; i < b.size();) {
            uint32_t r = static_cast<uint32_t>(next32());
            for (int n = 0; n < 4 && i < b.size(); ++n, r >>= 8) b[i++] = static_cast<unsigned char>(r);
        }
    }
};

struct Store {  // owns the bytes behind a list of direct buffers
    std::vector<std::vector<unsigned char>> mem;
    std::vector<ByteBuffer> bb;
    Store(int n, size_t len) : mem(n, std::vector<unsigned char>(len)), bb(n)
    {
        for (int i = 0; i < n; ++i) bb[i] = ByteBuffer::wrapDirect(mem[i].data(), len);
    }
    Buffers all() { Buffers b; for (auto& x : bb) b.push_back(&x); return b; }
};

static int cpu_checks()
{
    NativeRSEncoder enc(ErasureCoderOptions(4, 2));
    Store d(4, 16), p(2, 16), bad(1, 17);
    EXPECT(throws<ErasureCodeException>([&] { Buffers i = d.all(); i.pop_back(); enc.encode(i, p.all()); },
                                        "Invalid inputs length for encoding"));
    EXPECT(throws<ErasureCodeException>([&] { Buffers o = p.all(); o.push_back(&bad.bb[0]); enc.encode(d.all(), o); },
                                        "Invalid outputs length for encoding"));
    EXPECT(throws<ErasureCodeException>([&] { Buffers o{&p.bb[0], &bad.bb[0]}; enc.encode(d.all(), o); },
                                        "not of length 16"));
    EXPECT(throws<ErasureCodeException>([&] { enc.encode(Buffers(4, nullptr), p.all()); }, "all being null"));
    Store z(4, 0), zp(2, 0);
    enc.encode(z.all(), zp.all());  // zero length: no native call (JEC/ErasureEncoder.java:41-44)
    NativeRSDecoder dec(ErasureCoderOptions(4, 2));
    EXPECT(throws<ErasureCodeException>([&] { Buffers i = d.all(); i.pop_back(); dec.decode(i, {1, 2, 3}, {0}, {&p.bb[0]}); },
                                        "Invalid inputs length for decoding"));
    EXPECT(throws<ErasureCodeException>([&] { dec.decode(d.all(), {1, 2, 3, 4}, {0, 5}, {&p.bb[0]}); }, "mismatch"));
    EXPECT(throws<NullPointerException>([&] { dec.decode(d.all(), {1, 2, 3, 4}, {0}, {nullptr}); }));
    enc.release();
    EXPECT(throws<IOException>([&] { enc.encode(d.all(), p.all()); }, "NativeRSEncoder closed"));
    int ndev = 0;
    if (elect_ec_device_count(&ndev) != ELECT_EC_OK) {  // no device: compute fails loudly
        NativeRSEncoder e2(ErasureCoderOptions(4, 2));
        EXPECT(throws<DeviceError>([&] { e2.encode(d.all(), p.all()); }, "no HIP device"));
    }
    // checked device-batch calls: shapes and strides are checked before anything is
    // enqueued (no device needed; the pointers below are never dereferenced)
    {
        using elect::device::DeviceBatch;
        elect_ec_coder* c = nullptr;
        EXPECT(elect_ec_coder_create(4, 2, &c) == ELECT_EC_OK);
        alignas(16) static unsigned char fake[1];
        const DeviceBatch st = DeviceBatch::contiguous(fake, 16, 6, 64);
        const int dec[4] = {1, 2, 3, 4}, era[1] = {0}, era2[2] = {0, 5};
        auto bad = [&](auto&& f, const char* needle) { return throws<std::invalid_argument>(f, needle); };
        // a tiled view decoded into a buffer of another stripe count / length (round 2's fault)
        EXPECT(bad([&] { elect::device::decode_batch(c, st, dec, era, 1, DeviceBatch::contiguous(fake, 1, 1, 1024),
                                                     ELECT_EC_INPUTS_BY_UNIT, 0, nullptr); }, "outputs"));
        EXPECT(bad([&] { elect::device::decode_batch(c, st, dec, era2, 2, st.slice(0, 3),
                                                     ELECT_EC_INPUTS_BY_UNIT | ELECT_EC_OUTPUTS_BY_UNIT, 0, nullptr); },
                   "outputs"));
        EXPECT(bad([&] { elect::device::decode_batch(c, st.slice(0, 3), dec, era, 1,
                                                     DeviceBatch::contiguous(fake, 16, 1, 64), 0, 0, nullptr); },
                   "inputs"));
        EXPECT(bad([&] { elect::device::encode_batch(c, st.slice(0, 4), DeviceBatch::contiguous(fake, 8, 2, 64), nullptr); },
                   "parity"));
        EXPECT(bad([&] { elect::device::encode_batch(c, st.slice(0, 3), st.slice(4, 2), nullptr); }, "data"));
        // geometry right, but the strides run past the allocation
        DeviceBatch small = st;
        small.bytes = 16 * 6 * 64 - 1;
        EXPECT(bad([&] { elect::device::encode_batch(c, small.slice(0, 4), small.slice(4, 2), nullptr); }, "past"));
        EXPECT(bad([&] { elect::device::encode_update_batch(c, 0, st.slice(0, 1), st.slice(1, 1), st.slice(4, 2),
                                                            DeviceBatch::contiguous(fake, 16, 1, 64), nullptr); },
                   "parity_out"));
        // a well-formed call reaches the C ABI (which, without a device, fails loudly)
        int nd = 0;
        if (elect_ec_device_count(&nd) != ELECT_EC_OK)
            EXPECT(elect::device::encode_batch(c, st.slice(0, 4), st.slice(4, 2), nullptr) == ELECT_EC_ENODEV);
        elect_ec_coder_destroy(c);
    }
    return failures;
}

static void dump(const std::string& dir, const std::string& name, const std::vector<unsigned char>& v)
{
    std::ofstream f(dir + "/" + name, std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size()));
}

static int gpu_erasure_code_test(const std::string& out)
{
    const int k = 4, m = 2;
    const size_t L = 4099;
    JavaRandom random(123);
    NativeRSEncoder encoder(ErasureCoderOptions(k, m));
    NativeRSDecoder decoder(ErasureCoderOptions(k, m));
    Store data(k, L), modified(k, L), parity(m, L), second(m, L), upd(m, L), out1(1, L), out2(1, L);
    std::vector<unsigned char> tmp(L);
    for (int i = 0; i < k; ++i) {
        random.nextBytes(tmp);
        data.mem[i] = tmp;
        modified.mem[i] = tmp;
    }
    random.nextBytes(tmp);
    modified.mem[0] = tmp;
    encoder.encode(data.all(), parity.all());
    encoder.encode(modified.all(), second.all());
    decoder.decode({&parity.bb[0], &data.bb[1], &data.bb[2], &data.bb[3]}, {4, 1, 2, 3}, {0}, out1.all());
    decoder.decode({&second.bb[0], &modified.bb[1], &modified.bb[2], &modified.bb[3]}, {4, 1, 2, 3}, {0}, out2.all());
    encoder.encodeUpdate({&data.bb[0], &modified.bb[0], &parity.bb[0], &parity.bb[1]}, upd.all(), 0);
    EXPECT(out1.mem[0] == data.mem[0]);
    EXPECT(out2.mem[0] == modified.mem[0]);
    EXPECT(upd.mem[0] == second.mem[0] && upd.mem[1] == second.mem[1]);
    for (int i = 0; i < k; ++i) dump(out, "data" + std::to_string(i), data.mem[i]);
    for (int r = 0; r < m; ++r) {
        dump(out, "parity" + std::to_string(r), parity.mem[r]);
        dump(out, "second" + std::to_string(r), second.mem[r]);
        dump(out, "update" + std::to_string(r), upd.mem[r]);
    }
    return failures;
}

int main(int argc, char** argv)
{
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    const int rc = mode == "gpu" ? gpu_erasure_code_test(argc > 2 ? argv[2] : ".") : cpu_checks();
    std::printf("%s: %d failure(s)\n", mode.c_str(), rc);
    return rc == 0 ? 0 : 1;
}

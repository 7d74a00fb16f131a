// The host-memory path as a JVM process would drive it: no Python, no torch in
// the process, so libelect_ec.so runs on /opt/rocm's HIP / HSA runtime (the one
// it links), not on the copy PyTorch bundles.  T threads, each with
// its units back to back at odd offsets in one malloc'd block (so every unit
// has partial end pages and shares them with a neighbour), make every call
// ELECT's JNI methods make (encodeImpl, encodeExImpl with content lengths and
// hashes, decodeImpl, encodeUpdateImpl in place) at ELECT's codeLength, lone
// (thread 0 first, alone) and concurrently.  Each thread writes its inputs and
// outputs to <dir>/t<T>_<name>; tests/test_gpu_notorch.py checks them against
// the CPU oracle.  The library's own stats go to <dir>/stats.txt.
//
//   g++ -std=c++17 -O1 -I include tests/cpp/host_notorch.cpp -L elect_amd -lelect_ec
//       -Wl,-rpath,<repo>/elect_amd -pthread -o tests/cpp/host_notorch   (tests/test_gpu_notorch.py builds it)
//   tests/cpp/host_notorch <dir> [threads=4] [L=4404020]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "elect_ec.h"

namespace {

constexpr int kK = 4, kM = 2;

bool dump(const std::string& path, const unsigned char* p, size_t n)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, n, f) == n;
    return std::fclose(f) == 0 && ok;
}

// One caller's whole sequence; returns the number of failed calls.
int caller(const elect_ec_coder* coder, const std::string& dir, int t, size_t L)
{
    constexpr int kUnits = kK + kM + 2;  // data, parity, a rebuilt unit, a new-data unit
    constexpr size_t kGap = 21;
    std::vector<unsigned char> block(kUnits * (L + kGap) + 64);
    unsigned char* u[kUnits];
    for (int i = 0; i < kUnits; ++i) u[i] = block.data() + 1 + (t % 7) + i * (L + kGap);  // odd offsets
    std::mt19937_64 rng(1000 + t);
    for (int i = 0; i < kUnits; ++i)
        for (size_t b = 0; b < L; ++b) u[i][b] = static_cast<unsigned char>(rng());
    const unsigned char* data[kK] = {u[0], u[1], u[2], u[3]};
    unsigned char* parity[kM] = {u[4], u[5]};
    const std::string pre = dir + "/t" + std::to_string(t) + "_";
    int bad = 0;
    for (int j = 0; j < kK; ++j) bad += !dump(pre + "data" + std::to_string(j), u[j], L);
    bad += !dump(pre + "new", u[7], L);
    // encodeImpl
    bad += elect_ec_encode(coder, data, parity, L) != ELECT_EC_OK;
    for (int r = 0; r < kM; ++r) bad += !dump(pre + "parity" + std::to_string(r), parity[r], L);
    // decodeImpl: data unit 2 from parity 0 and data 0, 1, 3
    const unsigned char* surv[kK] = {u[4], u[0], u[1], u[3]};
    const int idx[kK] = {kK, 0, 1, 3}, erased[1] = {2};
    unsigned char* rebuilt[1] = {u[6]};
    bad += elect_ec_decode(coder, surv, idx, erased, 1, rebuilt, L, 0) != ELECT_EC_OK;
    bad += !dump(pre + "rebuilt2", u[6], L);
    // encodeExImpl: zero fill to codeLength + parity hashCode
    const size_t lens[kK] = {L / 3, L, L - 4097, L - 9};
    int32_t hashes[kM] = {};
    bad += elect_ec_encode_ex(coder, data, lens, parity, L, hashes) != ELECT_EC_OK;
    for (int r = 0; r < kM; ++r) bad += !dump(pre + "parity_ex" + std::to_string(r), parity[r], L);
    bad += !dump(pre + "hashes_ex", reinterpret_cast<const unsigned char*>(hashes), sizeof hashes);
    // encodeUpdateImpl in place on the plain parity: data unit 1 -> new
    bad += elect_ec_encode(coder, data, parity, L) != ELECT_EC_OK;
    const unsigned char* upd_in[2 + kM] = {u[1], u[7], u[4], u[5]};
    bad += elect_ec_encode_update(coder, upd_in, 1, parity, L) != ELECT_EC_OK;
    for (int r = 0; r < kM; ++r) bad += !dump(pre + "parity_upd" + std::to_string(r), parity[r], L);
    return bad;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    const int T = argc > 2 ? std::atoi(argv[2]) : 4;
    const size_t L = argc > 3 ? static_cast<size_t>(std::atoll(argv[3])) : 4404020;
    int ndev = 0;
    if (elect_ec_device_count(&ndev) != ELECT_EC_OK || ndev == 0) {
        std::printf("no device\n");
        return 3;
    }
    elect_ec_coder* coder = nullptr;
    if (elect_ec_coder_create(kK, kM, &coder) != ELECT_EC_OK) return 2;
    int bad = caller(coder, dir, 0, L);  // a lone caller first
    std::vector<int> fails(T, 0);
    std::vector<std::thread> th;
    for (int t = 1; t <= T; ++t) th.emplace_back([&, t] { fails[t - 1] = caller(coder, dir, t, L); });
    for (auto& x : th) x.join();
    for (int f : fails) bad += f;
    uint64_t st[19] = {};
    const int n = elect_ec_host_path_stats(st, 19);
    if (FILE* f = std::fopen((dir + "/stats.txt").c_str(), "w")) {
        for (int i = 0; i < n; ++i) std::fprintf(f, "%llu\n", static_cast<unsigned long long>(st[i]));
        std::fclose(f);
    }
    elect_ec_coder_destroy(coder);
    std::printf("%d failed call(s)\n", bad);
    return bad == 0 ? 0 : 1;
}

// Test infrastructure (tests/test_sanitized.py): a host-only driver of libastyle's C ABI, built
// with -fsanitize=address,undefined (tests/san/build.py) and run on the CPU.  It exercises the
// entry points that parse untrusted input or validate caller input without a GPU:
//   ckpt <list>        every prefix named in <list> (one per line) through ast_ckpt_open, then
//                      every entry through ast_ckpt_entry and ast_ckpt_read_f32 (the TF
//                      checkpoint-V2 reader of Saver.restore, methods.py:79-84); one line of
//                      return codes per prefix on stdout
//   cfg <seed> <n>     n seeded random ast_cfg values (in and out of range) through
//                      ast_workspace_bytes, the validation / sizing of ast_create
//                      (methods.py:44-77); one line per config
// A sanitizer report aborts the process (halt_on_error, -fno-sanitize-recover), so a clean exit
// means no report.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../../include/astyle.h"

static int run_ckpt(const char* list) {
    std::ifstream in(list);
    std::string pre;
    while (std::getline(in, pre)) {
        if (pre.empty()) continue;
        ast_ckpt* ck = nullptr;
        const int rc = ast_ckpt_open(pre.c_str(), &ck);
        int nread = 0, nfail = 0;
        if (rc == 0) {
            const int n = ast_ckpt_num_entries(ck);
            for (int i = 0; i < n; ++i) {
                char name[512];
                int dtype = 0, ndim = 0;
                int64_t dims[8];
                if (ast_ckpt_entry(ck, i, name, sizeof name, &dtype, &ndim, dims, 8)) { ++nfail; continue; }
                int64_t el = 1;
                bool ok = true;
                for (int k = 0; k < ndim; ++k) {
                    if (dims[k] < 0 || (dims[k] && el > (int64_t(1) << 26) / dims[k])) { ok = false; break; }
                    el *= dims[k];
                }
                if (!ok) { ++nfail; continue; }
                std::vector<float> buf((size_t)el + 1);
                if (ast_ckpt_read_f32(ck, name, buf.data(), (size_t)el) == 0) ++nread; else ++nfail;
                // a wrong element count must be refused
                if (ast_ckpt_read_f32(ck, name, buf.data(), (size_t)el + 1) == 0) { std::printf("BAD count accepted\n"); return 3; }
            }
            ast_ckpt_close(ck);
        }
        std::printf("%d %d %d\n", rc, nread, nfail);
    }
    return 0;
}

static int run_cfg(unsigned seed, int n) {
    std::mt19937 rng(seed);
    auto pick = [&](std::initializer_list<int> v) { return *(v.begin() + rng() % v.size()); };
    // mostly valid values (so the sizing paths run), now and then an invalid one
    auto mix = [&](std::initializer_list<int> ok, std::initializer_list<int> bad) {
        return rng() % 8 ? *(ok.begin() + rng() % ok.size()) : *(bad.begin() + rng() % bad.size());
    };
    for (int i = 0; i < n; ++i) {
        ast_cfg c;
        std::memset(&c, 0, sizeof c);
        c.batch = mix({1, 2, 7, 256, 2048, 1 << 20, 0x7fffffff}, {-3, 0});
        c.T = mix({512, 1024, 3584, 12800, 16384, 1 << 20, 0x7ffffe00}, {-512, 0, 1, 511, 1000});
        c.n_cont = mix({1, 2, 32}, {-1, 0, 33});
        c.n_style = mix({1, 10, 30, 32}, {-1, 0, 33});
        for (int k = 0; k < AST_MAX_TAPS; ++k) {
            c.cont_ids[k] = rng() % 64 ? pick({0, 9, 25, 29, 30, 31}) : pick({-1, 32, 1000});
            c.style_ids[k] = rng() % 64 ? pick({0, 3, 7, 29, 30}) : pick({-1, 31});
        }
        c.cnt_channels = mix({1, 16, 128, 4096}, {-1, 0});
        c.nb_channels = mix({1, 64, 128, 4096}, {-1, 0});
        c.gatys = pick({0, 1, 7});
        c.precision = mix({0, 1, 2}, {-1, 3});
        c.lambd = 100.f;
        size_t bytes = 0;
        const int rc = ast_workspace_bytes(&c, &bytes);
        std::printf("%d %zu\n", rc, rc ? (size_t)0 : bytes);
    }
    // null arguments
    if (ast_workspace_bytes(nullptr, nullptr) == 0) return 3;
    if (ast_ckpt_open(nullptr, nullptr) == 0) return 3;
    if (ast_ot_admm(nullptr, nullptr, 0, 0, 1, 1, 1e-4, 1e5, nullptr, nullptr, nullptr, nullptr) == 0) return 3;
    if (ast_ot_admm(nullptr, nullptr, 1, 1, 1, 1, 1e-4, 1e5, nullptr, nullptr, nullptr, nullptr) == 0) return 3;
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 3 && !std::strcmp(argv[1], "ckpt")) return run_ckpt(argv[2]);
    if (argc >= 4 && !std::strcmp(argv[1], "cfg")) return run_cfg((unsigned)std::atoi(argv[2]), std::atoi(argv[3]));
    std::fprintf(stderr, "usage: fuzz_driver ckpt <list> | cfg <seed> <n>\n");
    return 2;
}

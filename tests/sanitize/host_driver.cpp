// Host-side sanitizer driver for libcbw's runtime (no GPU): built by tools/sanitize_host.sh with runtime.cpp under
// AddressSanitizer + UndefinedBehaviorSanitizer (host code only: -Xarch_host), linked with the unsanitized kernel
// objects.  It runs the runtime's host-only code -- cbw_dtw (transformers' _dynamic_time_warping restated, the
// token-timestamp path, reference pba_whisper.py:333-336 via 4.37.2 generate) over many shapes, and the argument
// validation of every handle constructor and the launch wrappers that check before touching the device -- and
// checks the documented error codes.  A sanitizer report aborts the process (halt_on_error=1): exit != 0.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cbw.h"

static int failures = 0;
#define EXPECT(cond, what)                                                    \
    do {                                                                      \
        if (!(cond)) {                                                        \
            std::fprintf(stderr, "FAIL %s (%s:%d): %s\n", what, __FILE__, __LINE__, cbw_last_error()); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

// DTW path properties (size-independent): starts at (0, 0), ends at (rows-1, cols-1), every step advances text, time
// or both by exactly one, so the length lies in [max(rows, cols), rows + cols - 1]; and the path's cost is minimal
// among paths with those steps (checked against an independent f64 dynamic programme within f32 rounding).
static void check_dtw(int rows, int cols, std::mt19937& rng) {
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::vector<double> m((size_t)rows * cols);
    for (auto& v : m) v = u(rng);
    std::vector<int32_t> ti(rows + cols), tj(rows + cols);
    int n = -1;
    EXPECT(cbw_dtw(m.data(), rows, cols, ti.data(), tj.data(), &n) == CBW_OK, "cbw_dtw ok");
    EXPECT(n >= (rows > cols ? rows : cols) && n <= rows + cols - 1, "dtw length in range");
    if (n < 1) return;
    EXPECT(ti[0] == 0 && tj[0] == 0, "dtw starts at (0, 0)");
    EXPECT(ti[n - 1] == rows - 1 && tj[n - 1] == cols - 1, "dtw ends at the corner");
    double path = m[0];
    for (int k = 1; k < n; ++k) {
        const int di = ti[k] - ti[k - 1], dj = tj[k] - tj[k - 1];
        EXPECT((di == 0 || di == 1) && (dj == 0 || dj == 1) && (di + dj) > 0, "dtw unit steps");
        path += m[(size_t)ti[k] * cols + tj[k]];
    }
    std::vector<double> c((size_t)(rows + 1) * (cols + 1), 1e300);
    c[0] = 0.0;
    for (int i = 1; i <= rows; ++i)
        for (int j = 1; j <= cols; ++j) {
            double b = c[(size_t)(i - 1) * (cols + 1) + j - 1];
            b = std::min(b, c[(size_t)(i - 1) * (cols + 1) + j]);
            b = std::min(b, c[(size_t)i * (cols + 1) + j - 1]);
            c[(size_t)i * (cols + 1) + j] = m[(size_t)(i - 1) * cols + j - 1] + b;
        }
    const double best = c[(size_t)rows * (cols + 1) + cols];
    EXPECT(path <= best + 1e-4 * (rows + cols), "dtw path cost minimal (f32 tables)");
}

int main() {
    EXPECT(cbw_version() == 1, "cbw_version");
    EXPECT(cbw_last_error() != nullptr, "cbw_last_error");
    EXPECT(cbw_source_id() != nullptr && std::strlen(cbw_source_id()) == 16, "cbw_source_id");

    std::mt19937 rng(1234);
    const int shapes[][2] = {{1, 1}, {1, 7}, {7, 1}, {2, 2}, {3, 50}, {50, 3}, {17, 23}, {64, 1500}, {224, 1500}};
    for (auto& s : shapes) check_dtw(s[0], s[1], rng);
    for (int t = 0; t < 200; ++t) {
        std::uniform_int_distribution<int> d(1, 96);
        check_dtw(d(rng), d(rng), rng);
    }
    double one = 0.0;
    const float onef = 0.f;
    int32_t a = 0, b = 0;
    int n = 0;
    EXPECT(cbw_dtw(nullptr, 1, 1, &a, &b, &n) == CBW_ERR_INVALID, "dtw null matrix");
    EXPECT(cbw_dtw(&one, 0, 1, &a, &b, &n) == CBW_ERR_INVALID, "dtw zero rows");
    EXPECT(cbw_dtw(&one, 1, -3, &a, &b, &n) == CBW_ERR_INVALID, "dtw negative cols");
    EXPECT(cbw_dtw(&one, 1, 1, nullptr, &b, &n) == CBW_ERR_INVALID, "dtw null text_idx");

    // handle constructors: configuration checks come before any device call
    cbw_kws* kh = nullptr;
    EXPECT(cbw_kws_create(nullptr, &kh) == CBW_ERR_INVALID, "kws_create null cfg");
    cbw_kws_config kc{3, 1280, 2, 64, 50};
    EXPECT(cbw_kws_create(&kc, nullptr) == CBW_ERR_INVALID, "kws_create null out");
    cbw_kws_config bad = kc;
    bad.n_layers = 0;
    EXPECT(cbw_kws_create(&bad, &kh) == CBW_ERR_INVALID, "kws_create n_layers 0");
    bad = kc;
    bad.n_layers = 12;
    EXPECT(cbw_kws_create(&bad, &kh) == CBW_ERR_INVALID, "kws_create 12 layers with projection");
    bad = kc;
    bad.variant = 3;
    EXPECT(cbw_kws_create(&bad, &kh) == CBW_ERR_INVALID, "kws_create variant 3");
    bad = kc;
    bad.embedding_dim = 1000;
    EXPECT(cbw_kws_create(&bad, &kh) == CBW_ERR_INVALID, "kws_create D % 128");
    bad = kc;
    bad.variant = 0;
    bad.embedding_dim = 100;
    EXPECT(cbw_kws_create(&bad, &kh) == CBW_ERR_INVALID, "kws_create L variant D % 32");
    EXPECT(kh == nullptr, "kws_create leaves *out on failure");
    // a valid configuration reaches the device allocation: without a GPU it must fail cleanly (no leak, no crash)
    const int rc = cbw_kws_create(&kc, &kh);
    if (rc == CBW_OK) {
        EXPECT(cbw_kws_destroy(kh) == CBW_OK, "kws_destroy");
    } else {
        EXPECT(rc == CBW_ERR_HIP || rc == CBW_ERR_OOM, "kws_create without a GPU: a HIP / OOM error code");
        EXPECT(kh == nullptr, "kws_create leaves *out on device failure");
    }
    EXPECT(cbw_kws_destroy(nullptr) == CBW_OK, "kws_destroy null");
    EXPECT(cbw_kws_set_param(nullptr, "x", &onef, 0) == CBW_ERR_INVALID, "kws_set_param null handle");
    EXPECT(cbw_kws_finalize(nullptr) == CBW_ERR_INVALID, "kws_finalize null handle");
    EXPECT(cbw_kws_project_workspace_bytes(nullptr, 1, 1500) == -1, "kws_project_workspace_bytes null handle");

    cbw_encoder* eh = nullptr;
    EXPECT(cbw_encoder_create(nullptr, &eh) != CBW_OK, "encoder_create null cfg");
    cbw_encoder_config ebad{128, 1280, 0, 20, 5120};
    EXPECT(cbw_encoder_create(&ebad, &eh) != CBW_OK && eh == nullptr, "encoder_create 0 layers");
    ebad = {128, 1280, 32, 0, 5120};   // n_heads 0: rejected before d_model / n_heads (an integer division by zero)
    EXPECT(cbw_encoder_create(&ebad, &eh) == CBW_ERR_INVALID && eh == nullptr, "encoder_create 0 heads");
    EXPECT(cbw_encoder_set_param(nullptr, "x", &onef, 0) != CBW_OK, "encoder_set_param null handle");
    EXPECT(cbw_encoder_finalize(nullptr) != CBW_OK, "encoder_finalize null handle");

    cbw_decoder* dh = nullptr;
    EXPECT(cbw_decoder_create(nullptr, &dh) != CBW_OK, "decoder_create null cfg");
    cbw_decoder_config dbad{51866, 1280, 32, 20, 5120, 4096};
    EXPECT(cbw_decoder_create(&dbad, &dh) != CBW_OK && dh == nullptr, "decoder_create max_len > 448");
    dbad = {51866, 1280, 32, 0, 5120, 448};
    EXPECT(cbw_decoder_create(&dbad, &dh) == CBW_ERR_INVALID && dh == nullptr, "decoder_create 0 heads");
    EXPECT(cbw_decoder_vocab_padded(nullptr) == -1, "decoder_vocab_padded null handle");
    EXPECT(cbw_decoder_set_param(nullptr, "x", &onef, 0) != CBW_OK, "decoder_set_param null handle");

    // launch wrappers whose argument checks come before the device call (host pointers stand in: never dereferenced)
    float lg[4] = {0.f, 0.f, 0.f, 0.f}, pr[2] = {0.f, 0.f};
    int32_t ix[2] = {0, 0}, nn = 0;
    EXPECT(cbw_kws_spot(lg, nullptr, -1, 0.5f, 0, pr, ix, &nn, nullptr) == CBW_ERR_INVALID, "spot K < 0");
    EXPECT(cbw_kws_spot(nullptr, nullptr, 2, 0.5f, 0, pr, ix, &nn, nullptr) == CBW_ERR_INVALID, "spot null logits");
    EXPECT(cbw_kws_spot(lg, nullptr, 2, 0.5f, 0, pr, nullptr, &nn, nullptr) == CBW_ERR_INVALID, "spot null idx");
    EXPECT(cbw_kws_spot(lg, nullptr, 2, 0.5f, 7, pr, ix, &nn, nullptr) == CBW_ERR_INVALID, "spot mode 7");
    EXPECT(cbw_kws_band(lg, nullptr, 2, 0.5f, -0.1f, ix, &nn, nullptr) == CBW_ERR_INVALID, "band < 0");
    EXPECT(cbw_kws_band(lg, nullptr, 2, 0.5f, std::nanf(""), ix, &nn, nullptr) == CBW_ERR_INVALID, "band NaN");
    EXPECT(cbw_kws_band_scaled(lg, nullptr, 2, 0.5f, -1.f, ix, &nn, nullptr) == CBW_ERR_INVALID, "band_scaled coef < 0");
    uint64_t sum = 0;
    EXPECT(cbw_checksum(lg, 16, &sum, nullptr, 0, nullptr) == CBW_ERR_INVALID, "checksum null workspace");
    EXPECT(cbw_checksum((const char*)lg + 4, 8, &sum, lg, 1 << 20, nullptr) == CBW_ERR_INVALID, "checksum misaligned");
    EXPECT(cbw_checksum(lg, 16, &sum, lg, 0, nullptr) == CBW_ERR_OOM, "checksum workspace too small");

    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("host sanitizer driver: all checks passed\n");
    return 0;
}

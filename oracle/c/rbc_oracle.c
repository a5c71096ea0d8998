/* rbc_oracle.c — plain-C restatement of the RBC coding path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as the
 * checker at sizes too large for the numpy oracle, and by bench.py's
 * cpu_baseline leg as the "port" CPU baseline.  Never linked into the product.
 *
 * Restates:
 *   a1/a10  reed-solomon-erasure galois_8 + build_matrix  (GF(2^8), 0x11D, M = V·inv(V_top))
 *   a2      hbbft send_shards: BE u32 length prefix, zero pad, chunks of L
 *   a3      rse encode          parity[k] = XOR_j M[D+k][j] * data[j]
 *   a4/a5   hbbft MerkleTree::from_vec (SHA3 leaves, pair hash, odd promotion)
 *   a6      hbbft Proof::validate
 *   a7/a8   hbbft decode_from_shards + rse reconstruct (first D present rows) + glue_shards
 *   a9      tiny-keccak sha3_256 (FIPS-202)
 * all reached from /root/reference/src/hydrabadger/state.rs:484 (propose) and
 * state.rs:486-487 (handle_message).
 *
 * The GF inner loop has a scalar 64 KiB-table path and an AVX2 split-nibble
 * path (the algorithm of rse's simd-accel C backend), chosen at run time.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define ORC_OK 0
#define ORC_E_ARG (-1)
#define ORC_E_TOO_FEW_SHARDS_PRESENT (-2)
#define ORC_E_SINGULAR (-3)

/* ------------------------------------------------------------ GF(2^8) */
static uint8_t g_log[256], g_exp[510], g_mul[256][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_init(void) {
    unsigned b = 1;
    for (int l = 0; l < 255; ++l) {
        g_log[b] = (uint8_t)l;
        g_exp[l] = (uint8_t)b;
        g_exp[l + 255] = (uint8_t)b;
        b <<= 1;
        if (b >= 256) b ^= 0x11D;
    }
    for (int a = 0; a < 256; ++a)
        for (int c = 0; c < 256; ++c)
            g_mul[a][c] = (a && c) ? g_exp[g_log[a] + g_log[c]] : 0;
}
static inline uint8_t gmul(uint8_t a, uint8_t b) { return g_mul[a][b]; }
static uint8_t gexp(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return g_exp[(g_log[a] * n) % 255];
}
static uint8_t ginv(uint8_t a) { return g_exp[(255 - g_log[a]) % 255]; }

/* Gauss-Jordan inverse of n x n (row-major) in place into out. */
static int gf_invert(const uint8_t *m, int n, uint8_t *out) {
    uint8_t *a = (uint8_t *)malloc((size_t)n * 2 * n);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < 2 * n; ++c)
            a[r * 2 * n + c] = c < n ? m[r * n + c] : (uint8_t)(c - n == r);
    for (int r = 0; r < n; ++r) {
        uint8_t *row = a + r * 2 * n;
        if (row[r] == 0) {
            for (int rb = r + 1; rb < n; ++rb) {
                uint8_t *o = a + rb * 2 * n;
                if (o[r]) {
                    for (int c = 0; c < 2 * n; ++c) { uint8_t t = row[c]; row[c] = o[c]; o[c] = t; }
                    break;
                }
            }
        }
        if (row[r] == 0) { free(a); return ORC_E_SINGULAR; }
        if (row[r] != 1) {
            uint8_t s = ginv(row[r]);
            for (int c = 0; c < 2 * n; ++c) row[c] = gmul(s, row[c]);
        }
        for (int rb = 0; rb < n; ++rb) {
            if (rb == r) continue;
            uint8_t *o = a + rb * 2 * n;
            uint8_t s = o[r];
            if (s)
                for (int c = 0; c < 2 * n; ++c) o[c] ^= gmul(s, row[c]);
        }
    }
    for (int r = 0; r < n; ++r) memcpy(out + r * n, a + r * 2 * n + n, (size_t)n);
    free(a);
    return ORC_OK;
}

/* N x D coding matrix, row-major. */
int orc_build_matrix(uint32_t D, uint32_t Q, uint8_t *mat) {
    pthread_once(&g_once, gf_init);
    uint32_t N = D + Q;
    if (D == 0 || Q == 0 || N > 256) return ORC_E_ARG;
    uint8_t *v = (uint8_t *)malloc((size_t)N * D), *ti = (uint8_t *)malloc((size_t)D * D);
    for (uint32_t r = 0; r < N; ++r)
        for (uint32_t c = 0; c < D; ++c) v[r * D + c] = gexp((uint8_t)r, (int)c);
    int rc = gf_invert(v, (int)D, ti);
    if (rc == ORC_OK)
        for (uint32_t r = 0; r < N; ++r)
            for (uint32_t c = 0; c < D; ++c) {
                uint8_t acc = 0;
                for (uint32_t k = 0; k < D; ++k) acc ^= gmul(v[r * D + k], ti[k * D + c]);
                mat[r * D + c] = acc;
            }
    free(v);
    free(ti);
    return rc;
}

/* out ^= c * in over len bytes */
static void mac_scalar(uint8_t *out, const uint8_t *in, uint8_t c, uint64_t len) {
    const uint8_t *t = g_mul[c];
    for (uint64_t b = 0; b < len; ++b) out[b] ^= t[in[b]];
}

#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("avx2"))) static void mac_avx2(uint8_t *out, const uint8_t *in, uint8_t c,
                                                     uint64_t len) {
    uint8_t lo[16], hi[16];
    for (int x = 0; x < 16; ++x) { lo[x] = gmul(c, (uint8_t)x); hi[x] = gmul(c, (uint8_t)(x << 4)); }
    __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    __m256i m = _mm256_set1_epi8(0x0f);
    uint64_t b = 0;
    for (; b + 32 <= len; b += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(in + b));
        __m256i l = _mm256_shuffle_epi8(tl, _mm256_and_si256(x, m));
        __m256i h = _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi64(x, 4), m));
        __m256i o = _mm256_loadu_si256((const __m256i *)(out + b));
        _mm256_storeu_si256((__m256i *)(out + b), _mm256_xor_si256(o, _mm256_xor_si256(l, h)));
    }
    mac_scalar(out + b, in + b, c, len - b);
}
static int g_avx2 = -1;
static void mac(uint8_t *out, const uint8_t *in, uint8_t c, uint64_t len) {
    if (g_avx2 < 0) g_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
    if (c == 0) return;
    if (g_avx2) mac_avx2(out, in, c, len); else mac_scalar(out, in, c, len);
}
#else
static void mac(uint8_t *out, const uint8_t *in, uint8_t c, uint64_t len) {
    if (c) mac_scalar(out, in, c, len);
}
#endif

int orc_simd_enabled(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("avx2") ? 1 : 0;
#else
    return 0;
#endif
}

/* rse encode: shards [N][stride], data rows 0..D-1 read, parity rows written. */
int orc_rs_encode(uint32_t D, uint32_t Q, uint64_t L, uint8_t *shards, uint64_t stride) {
    uint32_t N = D + Q;
    if (D == 0 || Q == 0 || N > 256 || L == 0 || stride < L) return ORC_E_ARG;
    uint8_t *mat = (uint8_t *)malloc((size_t)N * D);
    int rc = orc_build_matrix(D, Q, mat);
    if (rc) { free(mat); return rc; }
    for (uint32_t k = 0; k < Q; ++k) {
        uint8_t *out = shards + (uint64_t)(D + k) * stride;
        memset(out, 0, L);
        for (uint32_t j = 0; j < D; ++j) mac(out, shards + (uint64_t)j * stride, mat[(D + k) * D + j], L);
    }
    free(mat);
    return ORC_OK;
}

/* rse reconstruct: present[N] (0/1); missing rows are (re)written. */
int orc_rs_reconstruct(uint32_t D, uint32_t Q, uint64_t L, uint8_t *shards, uint64_t stride,
                       const uint8_t *present) {
    uint32_t N = D + Q;
    if (D == 0 || Q == 0 || N > 256 || L == 0 || stride < L) return ORC_E_ARG;
    uint32_t np = 0, rows[256];
    for (uint32_t i = 0; i < N; ++i)
        if (present[i]) { if (np < D) rows[np] = i; ++np; }
    if (np == N) return ORC_OK;
    if (np < D) return ORC_E_TOO_FEW_SHARDS_PRESENT;
    uint8_t *mat = (uint8_t *)malloc((size_t)N * D), *sub = (uint8_t *)malloc((size_t)D * D),
            *dec = (uint8_t *)malloc((size_t)D * D);
    int rc = orc_build_matrix(D, Q, mat);
    if (!rc) {
        for (uint32_t r = 0; r < D; ++r) memcpy(sub + r * D, mat + rows[r] * D, D);
        rc = gf_invert(sub, (int)D, dec);
    }
    if (!rc) {
        for (uint32_t i = 0; i < D; ++i) {
            if (present[i]) continue;
            uint8_t *out = shards + (uint64_t)i * stride;
            memset(out, 0, L);
            for (uint32_t j = 0; j < D; ++j) mac(out, shards + (uint64_t)rows[j] * stride, dec[i * D + j], L);
        }
        for (uint32_t i = D; i < N; ++i) {
            if (present[i]) continue;
            uint8_t *out = shards + (uint64_t)i * stride;
            memset(out, 0, L);
            for (uint32_t j = 0; j < D; ++j) mac(out, shards + (uint64_t)j * stride, mat[i * D + j], L);
        }
    }
    free(mat); free(sub); free(dec);
    return rc;
}

/* ------------------------------------------------------------ Keccak / SHA3-256 */
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int ROTC[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#define ROL(x, n) ((n) ? (((x) << (n)) | ((x) >> (64 - (n)))) : (x))

static void keccakf(uint64_t a[25]) {
    for (int r = 0; r < 24; ++r) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ ROL(c[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = ROL(a[x + 5 * y], ROTC[x + 5 * y]);
        for (int y = 0; y < 5; ++y)
            for (int x = 0; x < 5; ++x)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= RC[r];
    }
}

void orc_sha3_256(const uint8_t *in, uint64_t len, uint8_t out[32]) {
    uint64_t a[25];
    memset(a, 0, sizeof a);
    const uint64_t rate = 136;
    while (len >= rate) {
        for (int i = 0; i < 17; ++i) { uint64_t w; memcpy(&w, in + 8 * i, 8); a[i] ^= w; }
        keccakf(a);
        in += rate;
        len -= rate;
    }
    uint8_t blk[136];
    memset(blk, 0, sizeof blk);
    memcpy(blk, in, len);
    blk[len] ^= 0x06;
    blk[rate - 1] ^= 0x80;
    for (int i = 0; i < 17; ++i) { uint64_t w; memcpy(&w, blk + 8 * i, 8); a[i] ^= w; }
    keccakf(a);
    memcpy(out, a, 32);
}

/* ------------------------------------------------------------ Merkle */
uint32_t orc_merkle_nodes(uint32_t n) {
    uint32_t t = 0;
    while (n > 1) { t += n; n = (n + 1) / 2; }
    return t + 1;
}

/* levels: flat digests level by level, root last ([nodes][32]). */
int orc_merkle_levels(uint32_t N, uint64_t L, const uint8_t *shards, uint64_t stride, uint8_t *levels) {
    if (N == 0) { orc_sha3_256(NULL, 0, levels); return ORC_OK; }
    for (uint32_t i = 0; i < N; ++i) orc_sha3_256(shards + (uint64_t)i * stride, L, levels + 32 * i);
    uint32_t base = 0, n = N;
    while (n > 1) {
        uint32_t nn = (n + 1) / 2;
        uint8_t *cur = levels + 32 * (uint64_t)base, *nxt = cur + 32 * (uint64_t)n;
        for (uint32_t k = 0; k < nn; ++k) {
            if (2 * k + 1 < n) orc_sha3_256(cur + 64 * k, 64, nxt + 32 * k);
            else memcpy(nxt + 32 * k, cur + 64 * k, 32);
        }
        base += n;
        n = nn;
    }
    return ORC_OK;
}

/* Proof::validate. digests[ndig][32]. returns 1 valid / 0 invalid. */
int orc_proof_validate(uint32_t n, const uint8_t *value, uint64_t L, uint32_t index, const uint8_t *digests,
                       uint32_t ndig, const uint8_t root[32]) {
    uint8_t d[32], pair[64];
    orc_sha3_256(value, L, d);
    uint32_t li = index, ln = n, used = 0;
    while (ln > 1) {
        if ((li ^ 1) < ln) {
            if (used >= ndig) return 0;
            const uint8_t *s = digests + 32 * used++;
            if (li & 1) { memcpy(pair, s, 32); memcpy(pair + 32, d, 32); }
            else { memcpy(pair, d, 32); memcpy(pair + 32, s, 32); }
            orc_sha3_256(pair, 64, d);
        }
        li /= 2;
        ln = (ln + 1) / 2;
    }
    if (used != ndig) return 0;
    return memcmp(d, root, 32) == 0;
}

/* ------------------------------------------------------------ synthetic inputs */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
void orc_synth_bytes(uint32_t tag, uint64_t instance, uint64_t nbytes, uint8_t *out) {
    uint64_t s = 0x48424247ULL ^ ((uint64_t)tag << 48) ^ instance;
    for (uint64_t k = 0; k < nbytes; k += 8) {
        uint64_t w = mix64(s + (k / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        uint64_t m = nbytes - k < 8 ? nbytes - k : 8;
        memcpy(out + k, &w, m);
    }
}

/* ------------------------------------------------------------ RBC glue */
static void num_shards(uint32_t N, uint32_t *D, uint32_t *Q) {
    uint32_t f = (N - 1) / 3;
    *Q = 2 * f;
    *D = N - *Q;
}
uint64_t orc_shard_len(uint32_t N, uint64_t P) {
    uint32_t D, Q;
    num_shards(N, &D, &Q);
    return (P + 4 + D - 1) / D;
}

/* send_shards for one instance: shards [N][stride], levels [nodes][32]. */
int orc_rbc_encode_merkle(uint32_t N, const uint8_t *payload, uint64_t P, uint8_t *shards, uint64_t stride,
                          uint8_t *levels) {
    uint32_t D, Q;
    if (N == 0 || N > 256) return ORC_E_ARG;
    num_shards(N, &D, &Q);
    uint64_t L = (P + 4 + D - 1) / D;
    if (stride < L) return ORC_E_ARG;
    /* value = BE u32 len || payload || zeros, chunked by L into rows of stride */
    uint8_t hdr[4] = {(uint8_t)(P >> 24), (uint8_t)(P >> 16), (uint8_t)(P >> 8), (uint8_t)P};
    for (uint32_t i = 0; i < N; ++i) {
        uint8_t *row = shards + (uint64_t)i * stride;
        for (uint64_t b = 0; b < L; ++b) {
            uint64_t v = (uint64_t)i * L + b;
            row[b] = v < 4 ? hdr[v] : (v - 4 < P ? payload[v - 4] : 0);
        }
    }
    if (Q) {
        int rc = orc_rs_encode(D, Q, L, shards, stride);
        if (rc) return rc;
    }
    return orc_merkle_levels(N, L, shards, stride, levels);
}

/* decode_from_shards + glue_shards for one instance.
 * status: 1 = Some(payload), 0 = None.  payload_out >= D*L bytes. */
int orc_rbc_decode(uint32_t N, uint64_t L, uint8_t *shards, uint64_t stride, const uint8_t *present,
                   const uint8_t root[32], uint8_t *payload_out, uint64_t *payload_len, uint8_t *status) {
    uint32_t D, Q;
    num_shards(N, &D, &Q);
    *status = 0;
    *payload_len = 0;
    if (Q) {
        int rc = orc_rs_reconstruct(D, Q, L, shards, stride, present);
        if (rc == ORC_E_TOO_FEW_SHARDS_PRESENT) return ORC_OK;
        if (rc) return rc;
    } else {
        for (uint32_t i = 0; i < N; ++i) if (!present[i]) return ORC_OK;
    }
    uint32_t nodes = orc_merkle_nodes(N);
    uint8_t *lv = (uint8_t *)malloc(32 * (size_t)nodes);
    orc_merkle_levels(N, L, shards, stride, lv);
    int same = memcmp(lv + 32 * (size_t)(nodes - 1), root, 32) == 0;
    free(lv);
    if (!same) return ORC_OK;
    uint64_t tot = (uint64_t)D * L;
    if (tot < 4) return ORC_OK;
    uint8_t h[4];
    for (int k = 0; k < 4; ++k) h[k] = shards[(uint64_t)(k / L) * stride + k % L];
    uint64_t len = ((uint64_t)h[0] << 24) | ((uint64_t)h[1] << 16) | ((uint64_t)h[2] << 8) | h[3];
    if (len > tot - 4) len = tot - 4;
    for (uint64_t k = 0; k < len; ++k) {
        uint64_t v = k + 4;
        payload_out[k] = shards[(v / L) * stride + v % L];
    }
    *payload_len = len;
    *status = 1;
    return ORC_OK;
}

/* ------------------------------------------------------------ threaded batch (cpu_baseline) */
typedef struct {
    uint32_t N;
    uint64_t P, L, stride, n, first, step;
    const uint8_t *payloads;
    uint8_t *shards, *levels;
    int rc;
} enc_job;

static void *enc_worker(void *arg) {
    enc_job *j = (enc_job *)arg;
    uint32_t nodes = orc_merkle_nodes(j->N);
    for (uint64_t i = j->first; i < j->n; i += j->step) {
        int rc = orc_rbc_encode_merkle(j->N, j->payloads + i * j->P, j->P,
                                       j->shards + i * j->N * j->stride, j->stride, j->levels + i * 32 * nodes);
        if (rc) j->rc = rc;
    }
    return NULL;
}

/* One instance per worker thread at a time (SURVEY.md §8(d) CPU baseline). */
int orc_rbc_encode_merkle_batch(uint32_t N, const uint8_t *payloads, uint64_t P, uint64_t n, uint8_t *shards,
                                uint64_t stride, uint8_t *levels, int threads) {
    pthread_once(&g_once, gf_init);
    if (threads < 1) threads = 1;
    pthread_t th[256];
    enc_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (enc_job){N, P, orc_shard_len(N, P), stride, n, (uint64_t)t, (uint64_t)threads,
                            payloads, shards, levels, 0};
        pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}

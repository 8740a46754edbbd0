/*
 * ec_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never shipped).
 *
 * A plain-C CPU restatement of the reference's built-in erasure codes, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg ONLY.  The
 * product (liberasurecode_amd/) never links, loads or calls this file.
 *
 * Parity pinning: this restatement is checked against
 *   - golden vectors produced by the reference's own liberasurecode_rs_vand.so.1 and
 *     libXorcode.so.1, compiled from /root/reference sources by oracle/Makefile into
 *     oracle/_ref/ (see tests/golden/make_golden.py), and
 *   - the reference unit tests' invariants (test/builtin/rs_vand/rs_galois_test.c:32-54,
 *     test/builtin/rs_vand/liberasurecode_rs_vand_test.c:62-294).
 *
 * What is restated (reference file:line):
 *   GF(2^16) log/antilog field, poly 0x1100b ........ src/builtin/rs_vand/rs_galois.c:38-117
 *   non-systematic Vandermonde + column reduction .... src/builtin/rs_vand/liberasurecode_rs_vand.c:139-289
 *   Gauss-Jordan inversion over GF(2^16) ............. liberasurecode_rs_vand.c:293-334
 *   region xor / multiply / dot product .............. liberasurecode_rs_vand.c:336-397
 *   encode / decode / reconstruct .................... liberasurecode_rs_vand.c:399-558
 *   fragment checksums: zlib crc32 (zlib 1.2.11, as called at src/erasurecode_postprocessing.c:
 *   66-67) and the legacy liberasurecode_crc32_alt .... src/utils/chksum/crc32.c:79-91
 * The flat-XOR HD codes are restated buffer-level in oracle/xor_oracle.py.
 *
 * One deliberate definition: for an odd blocksize the reference multiplies the trailing
 * byte through a signed `char` (liberasurecode_rs_vand.c:367-370), which indexes its log
 * table with a negative number for bytes >= 0x80 (undefined behaviour).  Here the trailing
 * byte is taken unsigned; for bytes < 0x80 this equals the reference.  The frontend always
 * passes an even blocksize (k*2 alignment, src/erasurecode_helpers.c:186-208).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ GF(2^16) ---- */

#define ORC_POLY 0x1100b
#define ORC_FIELD 65536
#define ORC_ORDER 65535

static int orc_log[ORC_FIELD];
static int orc_exp3[3 * ORC_ORDER]; /* antilog repeated three times */
static int *orc_exp = orc_exp3 + ORC_ORDER; /* centred: index range [-ORDER, 2*ORDER) */
static int orc_ready = 0;

void orc_gf_init(void)
{
    if (orc_ready)
        return;
    int v = 1;
    for (int e = 0; e < ORC_ORDER; e++) {
        orc_log[v] = e;
        orc_exp3[e] = v;
        orc_exp3[e + ORC_ORDER] = v;
        orc_exp3[e + 2 * ORC_ORDER] = v;
        v <<= 1;
        if (v & ORC_FIELD)
            v ^= ORC_POLY;
    }
    orc_ready = 1;
}

int orc_gf_mul(int a, int b)
{
    if (a == 0 || b == 0)
        return 0;
    return orc_exp[orc_log[a] + orc_log[b]];
}

int orc_gf_div(int a, int b)
{
    if (a == 0)
        return 0;
    if (b == 0)
        return -1;
    return orc_exp[orc_log[a] - orc_log[b]];
}

int orc_gf_inv(int a) { return orc_gf_div(1, a); }

/* log/antilog table digests, so tests can pin the tables themselves */
uint64_t orc_gf_table_digest(void)
{
    uint64_t h = 1469598103934665603ULL;
    for (int i = 1; i < ORC_FIELD; i++) {
        h = (h ^ (uint64_t)orc_log[i]) * 1099511628211ULL;
    }
    for (int i = 0; i < ORC_ORDER; i++) {
        h = (h ^ (uint64_t)orc_exp3[i]) * 1099511628211ULL;
    }
    return h;
}

/* ------------------------------------------------------- generator matrix ---- */

static void orc_swap_rows(int *a, int *b, int n)
{
    for (int c = 0; c < n; c++) {
        int t = a[c];
        a[c] = b[c];
        b[c] = t;
    }
}

/* Scale column `col` of rows [0, nrows) by `f`. */
static void orc_scale_col(int *mat, int ncols, int nrows, int col, int f)
{
    for (int r = 0; r < nrows; r++)
        mat[r * ncols + col] = orc_gf_mul(mat[r * ncols + col], f);
}

/* col[dst] ^= f * col[src] for rows [0, nrows). */
static void orc_axpy_col(int *mat, int ncols, int nrows, int src, int dst, int f)
{
    for (int r = 0; r < nrows; r++)
        mat[r * ncols + dst] ^= orc_gf_mul(mat[r * ncols + src], f);
}

static int orc_first_nonzero_at(int *mat, int ncols, int nrows, int col, int from_row)
{
    for (int r = from_row; r < nrows; r++)
        if (mat[r * ncols + col] != 0)
            return r;
    return -1;
}

/*
 * Systematic generator, (k+m) x k, row-major, written into `out`.
 * Same construction as make_systematic_matrix (liberasurecode_rs_vand.c:139-289):
 * rows r^0..r^(k-1) (row 0 = e0), column reduction of the top k x k to I,
 * then parity columns normalised so parity row 0 is all ones.
 */
int orc_rs_generator(int k, int m, int *out)
{
    int n = k + m;
    orc_gf_init();
    for (int c = 0; c < k; c++)
        out[c] = (c == 0);
    for (int r = 1; r < n; r++) {
        int p = 1;
        for (int c = 0; c < k; c++) {
            out[r * k + c] = p;
            p = orc_gf_mul(p, r);
        }
    }
    for (int d = 1; d < k; d++) {
        int piv = orc_first_nonzero_at(out, k, n, d, d);
        if (piv < 0)
            return -1;
        if (piv != d)
            orc_swap_rows(&out[piv * k], &out[d * k], k);
        if (out[d * k + d] != 1)
            orc_scale_col(out, k, n, d, orc_gf_inv(out[d * k + d]));
        for (int c = 0; c < k; c++) {
            int v = out[d * k + c];
            if (c != d && v != 0)
                orc_axpy_col(out, k, n, d, c, v);
        }
    }
    for (int c = 0; c < k; c++) {
        int v = out[k * k + c];
        if (v != 1)
            orc_scale_col(out + k * k, k, m, c, orc_gf_inv(v));
    }
    return 0;
}

/* ------------------------------------------------------- Gauss-Jordan ---- */

/* Inverse of the n x n matrix `a` (destroyed) into `inv`; gaussj_inversion, :293-334. */
int orc_gauss_inverse(int *a, int *inv, int n)
{
    memset(inv, 0, sizeof(int) * n * n);
    for (int i = 0; i < n; i++)
        inv[i * n + i] = 1;
    for (int i = 0; i < n; i++) {
        int piv = orc_first_nonzero_at(a, n, n, i, i);
        if (piv < 0)
            return -1;
        if (piv != i) {
            orc_swap_rows(&a[piv * n], &a[i * n], n);
            orc_swap_rows(&inv[piv * n], &inv[i * n], n);
        }
        if (a[i * n + i] != 1) {
            int f = orc_gf_inv(a[i * n + i]);
            for (int c = 0; c < n; c++) {
                a[i * n + c] = orc_gf_mul(a[i * n + c], f);
                inv[i * n + c] = orc_gf_mul(inv[i * n + c], f);
            }
        }
        for (int r = 0; r < n; r++) {
            if (r == i)
                continue;
            int f = a[r * n + i];
            for (int c = 0; c < n; c++) {
                a[r * n + c] ^= orc_gf_mul(a[i * n + c], f);
                inv[r * n + c] ^= orc_gf_mul(inv[i * n + c], f);
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------- region kernels ---- */

/* to ^= c * from over `bs` bytes of little-endian 16-bit words (region_multiply/xor). */
static void orc_region_madd(const uint8_t *from, uint8_t *to, int c, int bs)
{
    int words = bs / 2;
    if (c == 1) {
        for (int i = 0; i < bs; i++)
            to[i] ^= from[i];
        return;
    }
    if (c == 0)
        return;
    const uint16_t *f16 = (const uint16_t *)from;
    uint16_t *t16 = (uint16_t *)to;
    int lc = orc_log[c];
    for (int i = 0; i < words; i++) {
        int x = f16[i];
        if (x)
            t16[i] ^= (uint16_t)orc_exp[orc_log[x] + lc];
    }
    if (bs & 1) {
        int x = from[bs - 1];
        if (x)
            to[bs - 1] ^= (uint8_t)orc_exp[orc_log[x] + lc];
    }
}

/* out = sum_j row[j] * in[j]   (region_dot_product, :383-397) */
static void orc_dot(uint8_t *const *in, uint8_t *out, const int *row, int nin, int bs)
{
    memset(out, 0, bs);
    for (int j = 0; j < nin; j++)
        orc_region_madd(in[j], out, row[j], bs);
}

int orc_rs_encode(const int *G, uint8_t *const *data, uint8_t *const *parity, int k, int m, int bs)
{
    orc_gf_init();
    for (int p = 0; p < m; p++)
        orc_dot(data, parity[p], &G[(k + p) * k], k, bs);
    return 0;
}

/* Marks of the -1 terminated `missing` list into `flag[n]`; returns count. */
static int orc_flag_missing(const int *missing, int *flag, int n)
{
    int cnt = 0;
    memset(flag, 0, sizeof(int) * n);
    while (missing[cnt] > -1) {
        flag[missing[cnt]] = 1;
        cnt++;
    }
    return cnt;
}

/* First k present fragments in index order (data then parity): sources + G rows. */
static void orc_first_k(const int *G, uint8_t **data, uint8_t **parity, const int *flag, int k,
    int m, uint8_t **src, int *dec)
{
    int got = 0;
    for (int i = 0; i < k + m && got < k; i++) {
        if (flag[i])
            continue;
        src[got] = i < k ? data[i] : parity[i - k];
        memcpy(&dec[got * k], &G[i * k], sizeof(int) * k);
        got++;
    }
}

int orc_rs_decode(const int *G, uint8_t **data, uint8_t **parity, int k, int m, const int *missing,
    int bs, int rebuild_parity)
{
    int n = k + m;
    int flag[512];
    orc_gf_init();
    if (orc_flag_missing(missing, flag, n) > m)
        return -1;
    int *dec = (int *)malloc(sizeof(int) * k * k);
    int *inv = (int *)malloc(sizeof(int) * k * k);
    uint8_t **src = (uint8_t **)malloc(sizeof(uint8_t *) * k);
    orc_first_k(G, data, parity, flag, k, m, src, dec);
    orc_gauss_inverse(dec, inv, k);
    for (int i = 0; i < k; i++)
        if (flag[i])
            orc_dot(src, data[i], &inv[i * k], k, bs);
    if (rebuild_parity)
        for (int i = k; i < n; i++)
            if (flag[i])
                orc_dot(data, parity[i - k], &G[i * k], k, bs);
    free(dec);
    free(inv);
    free(src);
    return 0;
}

int orc_rs_reconstruct(const int *G, uint8_t **data, uint8_t **parity, int k, int m,
    const int *missing, int dest, int bs)
{
    int n = k + m;
    int flag[512];
    orc_gf_init();
    if (orc_flag_missing(missing, flag, n) > m)
        return -1;
    int *dec = (int *)malloc(sizeof(int) * k * k);
    int *inv = (int *)malloc(sizeof(int) * k * k);
    uint8_t **src = (uint8_t **)malloc(sizeof(uint8_t *) * k);
    orc_first_k(G, data, parity, flag, k, m, src, dec);
    orc_gauss_inverse(dec, inv, k);
    if (dest < k) {
        orc_dot(src, data[dest], &inv[dest * k], k, bs);
    } else {
        /* composite parity row over the first k available (:520-549) */
        int *row = (int *)calloc(k, sizeof(int));
        int j = 0;
        for (int d = 0; d < k; d++)
            if (!flag[d])
                row[j++] = G[dest * k + d];
        for (int t = 0; missing[t] > -1; t++) {
            int d = missing[t];
            if (d >= k)
                continue;
            for (int c = 0; c < k; c++)
                row[c] ^= orc_gf_mul(G[dest * k + d], inv[d * k + c]);
        }
        orc_dot(src, parity[dest - k], row, k, bs);
        free(row);
    }
    free(dec);
    free(inv);
    free(src);
    return 0;
}

/* ------------------------------------------------------- test data ---- */

/* splitmix64 byte stream: word i = mix(seed + (i+1)*golden), little-endian. */
void orc_splitmix_fill(uint64_t seed, uint8_t *out, int64_t nbytes)
{
    int64_t nw = nbytes / 8;
    for (int64_t i = 0; i <= nw; i++) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        for (int b = 0; b < 8; b++) {
            int64_t o = i * 8 + b;
            if (o < nbytes)
                out[o] = (uint8_t)(z >> (8 * b));
        }
    }
}

/* ------------------------------------------------------- checksums ---- */

static uint32_t orc_crc_tab[256];

static void orc_crc_init(void)
{
    if (orc_crc_tab[1])
        return;
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int b = 0; b < 8; b++)
            c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        orc_crc_tab[n] = c;
    }
}

/* zlib crc32(crc, buf, n): reflected CRC-32, polynomial 0xEDB88320, pre/post inversion. */
uint32_t orc_crc32(uint32_t crc, const uint8_t *buf, int64_t n)
{
    orc_crc_init();
    crc = ~crc;
    while (n--)
        crc = orc_crc_tab[(crc ^ *buf++) & 0xffu] ^ (crc >> 8);
    return ~crc;
}

/* liberasurecode_crc32_alt: the same table, but the 8-bit shift of the (signed) state keeps
 * bit 31 in the top byte (src/utils/chksum/crc32.c:86-88). */
uint32_t orc_crc32_alt(uint32_t crc, const uint8_t *buf, int64_t n)
{
    orc_crc_init();
    crc = ~crc;
    while (n--) {
        uint32_t sh = crc >> 8;
        if (crc & 0x80000000u)
            sh |= 0xff000000u;
        crc = orc_crc_tab[(crc ^ *buf++) & 0xffu] ^ sh;
    }
    return ~crc;
}

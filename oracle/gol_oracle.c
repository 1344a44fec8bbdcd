/*
 * gol_oracle.c -- CPU restatement of the reference generation step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libgol.so) never links,
 * loads or calls it; there is no CPU fallback in the product.
 *
 * PARITY UNPINNED: the reference (almendar/akka-game-of-life, Scala 2.11 /
 * Akka 2.3.9) ships no tests, fixtures or golden vectors, and it cannot be
 * built here (no JVM, no sbt, no Akka jars, no network).  This file restates
 * the reference algorithm line by line; it is cross-checked against an
 * independent numpy restatement (oracle/oracle.py) and against hand-derived
 * known-answer patterns (tests/test_oracle.py), not against reference output.
 *
 * Layout (shared with the device engine, DESIGN.md "Data layout"):
 *   - cell (x, y): row y, column x.  x = the reference's first coordinate i,
 *     y = the second coordinate j (BoardCreator.scala:47-53).
 *   - packed planes: row-major rows of `pitch` 32-bit words; cell x of a row
 *     is bit (x % 32) of word (x / 32), LSB first.  Bits at x >= W are zero.
 *
 * Topologies:
 *   ORACLE_TORUS       : neighbours wrap mod W and mod H (build-side topology
 *                        of BASELINE.json configs 2-5); the count is the
 *                        multiset sum over the 8 Moore offsets.
 *   ORACLE_REF_CLIPPED : the reference's geometry.  A board of size (w, h)
 *                        has (w+1) x (h+1) cells (BoardCreator.scala:47-53,
 *                        inclusive ranges) but neighbours are only taken from
 *                        [0,w) x [0,h) (package.scala:17-28, exclusive
 *                        ranges) -- so the caller passes W = w+1, H = h+1,
 *                        vis_w = w, vis_h = h.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_TORUS 0
#define ORACLE_REF_CLIPPED 1

#define ORACLE_MODE_MASKS 0
#define ORACLE_MODE_REF_EFFECTIVE 1

/* ------------------------------------------------------------------ */
/* Seeding: counter-based splitmix64, identical on host and device.     */
/* ------------------------------------------------------------------ */

uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static inline uint32_t row_tail_mask(int64_t W, int64_t word) {
    int64_t lo = word * 32;
    if (lo + 32 <= W) return 0xFFFFFFFFu;
    if (lo >= W) return 0u;
    return (uint32_t)((1ULL << (W - lo)) - 1ULL);
}

/* Word at global index i = y * wwords + c of a board W cells wide is
 *   hi32(splitmix64(seed + 0x9E3779B97F4A7C15 * (i + 1)))  &  tail mask.
 * This is the seeded stand-in for BoardCreator.scala:23's unseeded
 * Random.nextBoolean() per cell (Bernoulli(0.5)).  Fills rows
 * [row0, row0+rows) of the global board into `board` (local row 0 = row0). */
void oracle_seed_packed(uint32_t* board, int64_t W, int64_t row0, int64_t rows,
                        int64_t pitch, uint64_t seed) {
    int64_t wwords = (W + 31) / 32;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t c = 0; c < wwords; ++c) {
            uint64_t i = (uint64_t)(row0 + r) * (uint64_t)wwords + (uint64_t)c;
            uint64_t z = oracle_splitmix64(seed + 0x9E3779B97F4A7C15ULL * (i + 1));
            board[r * pitch + c] = (uint32_t)(z >> 32) & row_tail_mask(W, c);
        }
        for (int64_t c = wwords; c < pitch; ++c) board[r * pitch + c] = 0;
    }
}

/* java.util.Random-compatible initial board, the seeded analogue of
 * BoardCreator.scala:23:
 *   (generateAllCoordinates(boardSize) zip List.fill(n)(Random.nextBoolean())).toMap
 * generateAllCoordinates (BoardCreator.scala:47-53) yields (i, j) with i in
 * 0..w outer, j in 0..h inner, so the k-th nextBoolean() goes to
 * (x = k / (h+1), y = k % (h+1)).  java.util.Random(seed): 48-bit LCG,
 * nextBoolean() = next(1) != 0.  Output: cells[y * (w+1) + x] in {0,1}. */
void oracle_java_random_cells(uint8_t* cells, int w, int h, int64_t seed) {
    const uint64_t mult = 0x5DEECE66DULL, add = 0xBULL, mask = (1ULL << 48) - 1;
    uint64_t s = ((uint64_t)seed ^ mult) & mask;
    for (int i = 0; i <= w; ++i) {
        for (int j = 0; j <= h; ++j) {
            s = (s * mult + add) & mask;
            int bit = (int)(s >> 47); /* next(1) = (int)(seed >>> (48 - 1)) */
            cells[(int64_t)j * (w + 1) + i] = (uint8_t)(bit != 0);
        }
    }
}

/* ------------------------------------------------------------------ */
/* Scalar per-cell step: the literal restatement.                       */
/* ------------------------------------------------------------------ */

/* cells: uint8 [H][W], 0/1.
 *
 * Neighbourhood (package.scala:17-28): moves = List(-1,0,1); for i <- moves,
 * j <- moves: (x+i, y+j) if 0 <= x+i < w and 0 <= y+j < h and != (x, y).
 * Torus: offsets wrap mod W / H instead of being clipped.
 *
 * Rule (NextStateCellGathererActor.scala:39-46):
 *   mode MASKS         : n = number of live neighbours (multiset count);
 *                        new = cur ? (survive >> n) & 1 : (birth >> n) & 1.
 *                        B3/S23 is birth=0x008 survive=0x00C; the line-44
 *                        rule with a multiset count ("ref-literal") is
 *                        birth=0x000 survive=0x1F7.
 *   mode REF_EFFECTIVE : the rule exactly as it runs.  The gatherer holds a
 *                        Set[StateForEpoch] (one element per neighbour,
 *                        :12-18), line 42 maps it to Set[Boolean] (duplicates
 *                        collapse) and line 43 counts the `true`s, so
 *                        aliveNeighbours = 1 if any neighbour is alive else 0;
 *                        line 44: if (cur && aliveNeighbours == 3) !cur else cur.
 */
void oracle_step_cells(const uint8_t* cur, uint8_t* nxt, int64_t W, int64_t H,
                       int topology, int mode, uint32_t birth, uint32_t survive,
                       int64_t vis_w, int64_t vis_h) {
    for (int64_t y = 0; y < H; ++y) {
        for (int64_t x = 0; x < W; ++x) {
            int count = 0;
            int any_alive = 0;
            for (int i = -1; i <= 1; ++i) {
                for (int j = -1; j <= 1; ++j) {
                    int64_t nx = x + i, ny = y + j;
                    if (topology == ORACLE_TORUS) {
                        if (i == 0 && j == 0) continue;
                        nx = ((nx % W) + W) % W;
                        ny = ((ny % H) + H) % H;
                    } else {
                        if (!(nx >= 0 && nx < vis_w)) continue;  /* 0 until w contains newX */
                        if (!(ny >= 0 && ny < vis_h)) continue;  /* 0 until h contains newY */
                        if (nx == x && ny == y) continue;        /* (newX,newY) != (x,y)   */
                    }
                    int v = cur[ny * W + nx] ? 1 : 0;
                    count += v;
                    any_alive |= v;
                }
            }
            int c = cur[y * W + x] ? 1 : 0;
            int n;
            if (mode == ORACLE_MODE_REF_EFFECTIVE) {
                int alive_neighbours = any_alive; /* Set[Boolean] collapse, :42-43 */
                n = (c && alive_neighbours == 3) ? !c : c; /* :44 */
            } else {
                n = c ? (int)((survive >> count) & 1u) : (int)((birth >> count) & 1u);
            }
            nxt[y * W + x] = (uint8_t)n;
        }
    }
}

/* ------------------------------------------------------------------ */
/* Bit-packed, bit-sliced multithreaded step (also the CPU baseline).   */
/* ------------------------------------------------------------------ */

static inline uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

/* One output row from the visible rows above (a), centre (cv), below (b),
 * the real centre row (alive) and per-row scratch.  wrap: torus in x. */
static void packed_row(const uint32_t* a, const uint32_t* cv, const uint32_t* b,
                       const uint32_t* alive, uint32_t* out, int64_t wwords, int wrap,
                       uint32_t birth, uint32_t survive, int64_t W,
                       uint32_t* v0, uint32_t* v1) {
    /* vertical 3-sum per column: (v1 v0) = a + cv + b */
    for (int64_t j = 0; j < wwords; ++j) {
        uint32_t t = a[j] ^ cv[j];
        v0[j] = t ^ b[j];
        v1[j] = bfi32(t, b[j], a[j]); /* majority */
    }
    const int life = wrap && (birth == 0x8u && survive == 0xCu); /* needs centre visible */
    uint32_t Bm[9], Sm[9];
    for (int k = 0; k < 9; ++k) {
        Bm[k] = ((birth >> k) & 1u) ? 0xFFFFFFFFu : 0u;
        Sm[k] = ((survive >> k) & 1u) ? 0xFFFFFFFFu : 0u;
    }
    for (int64_t j = 0; j < wwords; ++j) {
        uint32_t p0, p1, n0, n1; /* previous / next word's column sums */
        if (j > 0) { p0 = v0[j - 1]; p1 = v1[j - 1]; }
        else if (wrap) { p0 = v0[wwords - 1]; p1 = v1[wwords - 1]; }
        else { p0 = 0; p1 = 0; }
        if (j + 1 < wwords) { n0 = v0[j + 1]; n1 = v1[j + 1]; }
        else if (wrap) { n0 = v0[0]; n1 = v1[0]; }
        else { n0 = 0; n1 = 0; }
        uint32_t w0 = (v0[j] << 1) | (p0 >> 31), e0 = (v0[j] >> 1) | (n0 << 31);
        uint32_t w1 = (v1[j] << 1) | (p1 >> 31), e1 = (v1[j] >> 1) | (n1 << 31);
        /* box sum T9 = (w1 w0) + (v1 v0) + (e1 e0), bits s3 s2 s1 s0 */
        uint32_t t0 = w0 ^ v0[j];
        uint32_t s0 = t0 ^ e0;
        uint32_t c0 = bfi32(t0, e0, w0);
        uint32_t t1 = w1 ^ v1[j];
        uint32_t p = t1 ^ e1;
        uint32_t q = bfi32(t1, e1, w1);
        uint32_t s1 = p ^ c0;
        uint32_t r2 = p & c0;
        uint32_t s2 = q ^ r2;
        uint32_t s3 = q & r2;
        uint32_t al = alive[j];
        uint32_t res;
        if (life) {
            res = bfi32(s2, al & ~(s1 | s0), s1 & s0);
        } else {
            /* n = T9 - centre_visible */
            uint32_t c = cv[j];
            uint32_t nn0 = s0 ^ c, b0 = c & ~s0;
            uint32_t nn1 = s1 ^ b0, b1 = b0 & ~s1;
            uint32_t nn2 = s2 ^ b1, b2 = b1 & ~s2;
            uint32_t nn3 = s3 ^ b2;
            uint32_t L[9];
            for (int k = 0; k < 9; ++k) L[k] = bfi32(al, Sm[k], Bm[k]);
            uint32_t m01 = bfi32(nn0, L[1], L[0]), m23 = bfi32(nn0, L[3], L[2]);
            uint32_t m45 = bfi32(nn0, L[5], L[4]), m67 = bfi32(nn0, L[7], L[6]);
            uint32_t m03 = bfi32(nn1, m23, m01), m47 = bfi32(nn1, m67, m45);
            uint32_t m07 = bfi32(nn2, m47, m03);
            res = bfi32(nn3, L[8], m07);
        }
        out[j] = res & row_tail_mask(W, j);
    }
}

/* cur/nxt: packed [H][pitch].  For ORACLE_REF_CLIPPED, neighbour rows
 * y >= vis_h and columns x >= vis_w are invisible (read as dead).
 * nthreads <= 0: OpenMP default. */
void oracle_step_packed(const uint32_t* cur, uint32_t* nxt, int64_t W, int64_t H,
                        int64_t pitch, int topology, uint32_t birth, uint32_t survive,
                        int64_t vis_w, int64_t vis_h, int nthreads) {
    const int64_t wwords = (W + 31) / 32;
    const int torus = (topology == ORACLE_TORUS);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        uint32_t* scratch = (uint32_t*)calloc((size_t)(7 * wwords + 8), sizeof(uint32_t));
        uint32_t* v0 = scratch;
        uint32_t* v1 = scratch + wwords;
        uint32_t* ma = scratch + 2 * wwords; /* masked copies for clipped mode */
        uint32_t* mc = scratch + 3 * wwords;
        uint32_t* mb = scratch + 4 * wwords;
        uint32_t* zero = scratch + 5 * wwords;
        uint32_t* vmask = scratch + 6 * wwords;
        for (int64_t j = 0; j < wwords; ++j) vmask[j] = row_tail_mask(torus ? W : vis_w, j);
#pragma omp for schedule(static)
        for (int64_t y = 0; y < H; ++y) {
            const uint32_t *a, *c, *b;
            const uint32_t* al = cur + y * pitch;
            if (torus) {
                a = cur + ((y + H - 1) % H) * pitch;
                c = al;
                b = cur + ((y + 1) % H) * pitch;
            } else {
                const uint32_t* src[3] = {y >= 1 ? cur + (y - 1) * pitch : zero, al,
                                          y + 1 < H ? cur + (y + 1) * pitch : zero};
                int64_t ys[3] = {y - 1, y, y + 1};
                uint32_t* dst[3] = {ma, mc, mb};
                for (int k = 0; k < 3; ++k) {
                    int vis = ys[k] >= 0 && ys[k] < vis_h && ys[k] < H;
                    for (int64_t j = 0; j < wwords; ++j) dst[k][j] = vis ? (src[k][j] & vmask[j]) : 0u;
                }
                a = ma; c = mc; b = mb;
            }
            packed_row(a, c, b, al, nxt + y * pitch, wwords, torus, birth, survive, W, v0, v1);
            for (int64_t j = wwords; j < pitch; ++j) nxt[y * pitch + j] = 0;
        }
        free(scratch);
    }
}

/* ------------------------------------------------------------------ */
/* State hash (sharding-invariant, order-independent).                  */
/* ------------------------------------------------------------------ */

/* The hash is a function of the logical board alone:
 * it reads the cells through the canonical group words below, whatever
 * layout, topology, shard decomposition or environment produced them. */

static uint32_t even_bits(uint32_t x) { /* bits 0, 2, .., 30 -> bits 0 .. 15 */
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}

/* Row-major pair (w0 = columns 0..31, w1 = 32..63) -> (even, odd) words. */
void oracle_to_pairs(uint32_t w0, uint32_t w1, uint32_t* e, uint32_t* o) {
    *e = even_bits(w0) | (even_bits(w1) << 16);
    *o = even_bits(w0 >> 1) | (even_bits(w1 >> 1) << 16);
}

/* Canonical words of column group g of a row-major row of `wwords` words:
 * the group is columns 64g .. 64g + 63, E holds its even columns (bit b =
 * column 64g + 2b), O its odd ones (bit b = column 64g + 2b + 1).  A row
 * with an odd number of words ends in a half group (its upper 16 bits 0). */
void oracle_canonical_words(const uint32_t* row, int64_t wwords, int64_t g, uint32_t* e, uint32_t* o) {
    const uint32_t w1 = 2 * g + 1 < wwords ? row[2 * g + 1] : 0u;
    oracle_to_pairs(row[2 * g], w1, e, o);
}

/* Keys of the state hash (DESIGN.md "State hash"; gol_kernels.h).  The
 * canonical words E, O of column group g of global row y contribute
 *   (E * A(y, 0) + O * A(y, 1)) * B(g)     (mod 2^64),
 *   A(y, 0) = ((t ^ (t >> 15)) << 1) | 1,  t = y * 0x9E3779B1   (mod 2^32)
 *   A(y, 1) = A(y, 0) + 0x6A09E666         (mod 2^32)
 *   B(g)    = fmix32(g + 0x7F4A7C15) | 1  (murmur3's 32-bit finaliser).
 * Both keys are odd, so (A * B) is odd and any single-word difference changes
 * the sum; a sum commutes, so the value is the same for one shard or many and
 * for any evaluation order. */
uint32_t oracle_hash_row_key(int64_t y, int odd) {
    uint32_t t = (uint32_t)y * 0x9E3779B1u;
    uint32_t a = ((t ^ (t >> 15)) << 1) | 1u;
    return odd ? a + 0x6A09E666u : a;
}

uint32_t oracle_hash_pair_key(uint32_t k) {
    uint32_t h = k + 0x7F4A7C15u;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h | 1u;
}

/* Rows [row0, row0+rows) of a row-major board with `wwords` words per row. */
uint64_t oracle_hash_packed(const uint32_t* board, int64_t wwords, int64_t row0, int64_t rows,
                            int64_t pitch) {
    const int64_t groups = (wwords + 1) / 2;
    uint64_t h = 0;
    /* a sum mod 2^64 commutes: rows in parallel give the same value */
#pragma omp parallel for schedule(static) reduction(+ : h) if (rows * wwords > (1 << 20))
    for (int64_t r = 0; r < rows; ++r) {
        const uint32_t a0 = oracle_hash_row_key(row0 + r, 0), a1 = oracle_hash_row_key(row0 + r, 1);
        for (int64_t g = 0; g < groups; ++g) {
            uint32_t e, o;
            oracle_canonical_words(board + r * pitch, wwords, g, &e, &o);
            const uint64_t b = oracle_hash_pair_key((uint32_t)g);
            h += ((uint64_t)e * a0 + (uint64_t)o * a1) * b;
        }
    }
    return h;
}

/* Multithreaded n-generation run with per-generation hashes (hashes may be
 * NULL).  Ping-pongs between `board` and `tmp`; the final state ends in
 * `board`.  Used for golden vectors and the CPU baseline. */
void oracle_run_packed(uint32_t* board, uint32_t* tmp, int64_t W, int64_t H, int64_t pitch,
                       int topology, uint32_t birth, uint32_t survive, int64_t vis_w,
                       int64_t vis_h, int64_t gens, uint64_t* hashes, int nthreads) {
    const int64_t wwords = (W + 31) / 32;
    uint32_t* a = board;
    uint32_t* b = tmp;
    for (int64_t g = 0; g < gens; ++g) {
        oracle_step_packed(a, b, W, H, pitch, topology, birth, survive, vis_w, vis_h, nthreads);
        if (hashes) hashes[g] = oracle_hash_packed(b, wwords, 0, H, pitch);
        uint32_t* t = a; a = b; b = t;
    }
    if (a != board) memcpy(board, a, (size_t)(H * pitch) * sizeof(uint32_t));
}

/* Pack / unpack between uint8 cells [H][W] and packed [H][pitch]. */
void oracle_pack(const uint8_t* cells, uint32_t* packed, int64_t W, int64_t H, int64_t pitch) {
    memset(packed, 0, (size_t)(H * pitch) * sizeof(uint32_t));
    for (int64_t y = 0; y < H; ++y)
        for (int64_t x = 0; x < W; ++x)
            if (cells[y * W + x]) packed[y * pitch + x / 32] |= 1u << (x % 32);
}

void oracle_unpack(const uint32_t* packed, uint8_t* cells, int64_t W, int64_t H, int64_t pitch) {
    for (int64_t y = 0; y < H; ++y)
        for (int64_t x = 0; x < W; ++x)
            cells[y * W + x] = (uint8_t)((packed[y * pitch + x / 32] >> (x % 32)) & 1u);
}

// K=3 shared encodings of the pair sum a+b (a,b 2-bit row sums), then T-gate tails
// over (3 code planes, x0, x1, c).
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef uint64_t u64; typedef uint16_t u16;
static u64 gate64(u64 a, u64 b, u64 c, int f) {
  u64 r = 0;
  for (int m = 0; m < 8; m++) if (f >> m & 1) r |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
  return r;
}
static u64 IN[6], CARE, TGT;
static int func_of(const u64* s, int k) {
  u64 stack[64]; int n = 1; stack[0] = CARE;
  for (int i = 0; i < k; i++) {
    int nn = 0; u64 tmp[64];
    for (int j = 0; j < n; j++) {
      u64 a = stack[j] & s[i], b = stack[j] & ~s[i];
      if ((a & TGT) && (a & ~TGT)) tmp[nn++] = a;
      if ((b & TGT) && (b & ~TGT)) tmp[nn++] = b;
    }
    n = nn; memcpy(stack, tmp, n * sizeof(u64));
    if (!n) return 1;
  }
  return 0;
}
static u64 canon(u64 t) { u64 a = t & CARE, b = ~t & CARE; return a < b ? a : b; }
// T=3 search with the globals set; returns 1 if found
static int t3(int verbose) {
  u64 G1[6000]; int n1 = 0;
  for (int i = 0; i < 6; i++) for (int j = i + 1; j < 6; j++) for (int k = j + 1; k < 6; k++)
    for (int f = 0; f < 256; f++) {
      u64 t = gate64(IN[i], IN[j], IN[k], f), c = canon(t);
      if (!c) continue;
      int dup = 0;
      for (int q = 0; q < 6 && !dup; q++) dup = canon(IN[q]) == c;
      for (int q = 0; q < n1 && !dup; q++) dup = canon(G1[q]) == c;
      if (!dup) G1[n1++] = t;
    }
  for (int a = 0; a < n1; a++) {
    u64 sig[8]; memcpy(sig, IN, sizeof IN); sig[6] = G1[a];
    for (int i = 0; i < 7; i++) for (int j = i + 1; j < 7; j++) for (int k = j + 1; k < 7; k++)
      for (int f = 0; f < 256; f++) {
        u64 t = gate64(sig[i], sig[j], sig[k], f);
        for (int x = 0; x < 7; x++) for (int y = x + 1; y < 7; y++) {
          u64 s3[3] = {sig[x], sig[y], t};
          if (func_of(s3, 3)) { if (verbose) printf("  T3 g1=%llx g2=(%d,%d,%d,%02x) fin(%d,%d)\n", (unsigned long long)G1[a], i, j, k, f, x, y); return 1; }
        }
      }
  }
  return 0;
}
static int t4(int verbose) {
  u64 G1[6000]; int n1 = 0;
  for (int i = 0; i < 6; i++) for (int j = i + 1; j < 6; j++) for (int k = j + 1; k < 6; k++)
    for (int f = 0; f < 256; f++) {
      u64 t = gate64(IN[i], IN[j], IN[k], f), c = canon(t);
      if (!c) continue;
      int dup = 0;
      for (int q = 0; q < 6 && !dup; q++) dup = canon(IN[q]) == c;
      for (int q = 0; q < n1 && !dup; q++) dup = canon(G1[q]) == c;
      if (!dup) G1[n1++] = t;
    }
  volatile int found = 0;
#pragma omp parallel for schedule(dynamic)
  for (int a = 0; a < n1; a++) {
    if (found) continue;
    u64 sig[8]; memcpy(sig, IN, sizeof IN); sig[6] = G1[a];
    for (int i = 0; i < 7; i++) for (int j = i + 1; j < 7; j++) for (int k = j + 1; k < 7; k++)
      for (int f = 0; f < 256; f++) {
        u64 t = gate64(sig[i], sig[j], sig[k], f);
        for (int x = 0; x < 7; x++) for (int y = x + 1; y < 7; y++) for (int z = y + 1; z < 7; z++) for (int w = z + 1; w < 7; w++) {
          u64 s5[5] = {t, sig[x], sig[y], sig[z], sig[w]};
          if (!func_of(s5, 5)) continue;
          for (int m = 0; m < 32; m++) {
            if (__builtin_popcount(m) != 3) continue;
            u64 s[3], yz[2]; int ns = 0, ny = 0;
            for (int b = 0; b < 5; b++) if (m >> b & 1) s[ns++] = s5[b]; else yz[ny++] = s5[b];
            for (int flips = 0; flips < 16; flips++) {
              int need[8]; for (int q = 0; q < 8; q++) need[q] = -1;
              int ok = 1;
              for (int r = 0; r < 64 && ok; r++) {
                if (!(CARE >> r & 1)) continue;
                int cls = (int)(yz[0] >> r & 1) | (int)(yz[1] >> r & 1) << 1;
                u64 cm = CARE & ((cls & 1) ? yz[0] : ~yz[0]) & ((cls & 2) ? yz[1] : ~yz[1]);
                if (!(cm & TGT) || !(cm & ~TGT)) continue;
                int pat = (int)(s[0] >> r & 1) << 2 | (int)(s[1] >> r & 1) << 1 | (int)(s[2] >> r & 1);
                int v = (int)(TGT >> r & 1) ^ (flips >> cls & 1);
                if (need[pat] < 0) need[pat] = v; else if (need[pat] != v) ok = 0;
              }
              if (ok) {
                if (verbose) {
#pragma omp critical
                  printf("  T4 g1=%llx g2=(%d,%d,%d,%02x) subset=(%d,%d,%d,%d) m=%x flips=%x\n", (unsigned long long)G1[a], i, j, k, f, x, y, z, w, m, flips);
                }
                found = 1; goto out;
              }
            }
          }
        }
      }
  out:;
  }
  return found;
}
int main(int argc, char** argv) {
  int want_t4 = argc > 1;
  // 4 inputs a0 a1 b0 b1: row r = a0 | a1<<1 | b0<<2 | b1<<3
  u16 I4[4] = {0};
  for (int r = 0; r < 16; r++) for (int i = 0; i < 4; i++) if (r >> i & 1) I4[i] |= 1 << r;
  int sumr[16]; for (int r = 0; r < 16; r++) sumr[r] = (r & 3) + (r >> 2);
  // enumerate distinct 16-bit functions reachable by 1 gate, then triples g1,g2,g3
  // store encodings as canonical code->class maps
  static unsigned char seen[1 << 24]; // hash of map
  long nenc = 0, ntried = 0, nfound = 0;
  for (int i1 = 0; i1 < 4; i1++) for (int j1 = i1 + 1; j1 < 4; j1++) for (int k1 = j1 + 1; k1 < 4; k1++) for (int f1 = 0; f1 < 256; f1++) {
    u16 g1 = (u16)gate64(I4[i1], I4[j1], I4[k1], f1);
    u16 s2[5] = {I4[0], I4[1], I4[2], I4[3], g1};
    for (int i2 = 0; i2 < 5; i2++) for (int j2 = i2 + 1; j2 < 5; j2++) for (int k2 = j2 + 1; k2 < 5; k2++) for (int f2 = 0; f2 < 256; f2++) {
      u16 g2 = (u16)gate64(s2[i2], s2[j2], s2[k2], f2);
      u16 s3[6] = {I4[0], I4[1], I4[2], I4[3], g1, g2};
      for (int i3 = 0; i3 < 6; i3++) for (int j3 = i3 + 1; j3 < 6; j3++) for (int k3 = j3 + 1; k3 < 6; k3++) for (int f3 = 0; f3 < 256; f3++) {
        u16 g3 = (u16)gate64(s3[i3], s3[j3], s3[k3], f3);
        // code map: code -> class bitset (classes 0..4, 5 = >=5)
        int cls[8] = {0};
        for (int r = 0; r < 16; r++) {
          int code = (g1 >> r & 1) | (g2 >> r & 1) << 1 | (g3 >> r & 1) << 2;
          int s = sumr[r] >= 5 ? 5 : sumr[r];
          cls[code] |= 1 << s;
        }
        int ok = 1;
        for (int c = 0; c < 8; c++) if (cls[c] & (cls[c] - 1)) ok = 0;
        if (!ok) continue;
        // canonical over 48 transforms: min of encoded map
        unsigned best = ~0u;
        int perm[6][3] = {{0,1,2},{0,2,1},{1,0,2},{1,2,0},{2,0,1},{2,1,0}};
        for (int p = 0; p < 6; p++) for (int fl = 0; fl < 8; fl++) {
          unsigned key = 0;
          for (int c = 0; c < 8; c++) {
            int b[3] = {c & 1, c >> 1 & 1, c >> 2 & 1}, nc = 0;
            for (int q = 0; q < 3; q++) nc |= (b[perm[p][q]] ^ (fl >> q & 1)) << q;
            int v = cls[c] ? __builtin_ctz(cls[c]) + 1 : 0;
            key = key * 0 + key; key |= (unsigned)v << (3 * nc);
          }
          if (key < best) best = key;
        }
        unsigned h = best & ((1u << 24) - 1);
        if (seen[h]) continue;
        seen[h] = 1;
        nenc++;
        // set up tail problem: rows bit0..2 code, 3..4 X, 5 c
        memset(IN, 0, sizeof IN); CARE = TGT = 0;
        for (int r = 0; r < 64; r++) {
          for (int i = 0; i < 6; i++) if (r >> i & 1) IN[i] |= 1ull << r;
          int code = r & 7, X = r >> 3 & 3, c = r >> 5 & 1;
          if (!cls[code]) continue;
          int s = __builtin_ctz(cls[code]);
          if (c && s == 0) continue;
          CARE |= 1ull << r;
          int S = s + X;
          if (S == 3 || (S == 4 && c)) TGT |= 1ull << r;
        }
        ntried++;
        int f = want_t4 ? t4(0) : t3(0);
        if (f) {
          nfound++;
          printf("enc g1=(%d%d%d,%02x)=%04x g2=(%d%d%d,%02x)=%04x g3=(%d%d%d,%02x)=%04x map:", i1, j1, k1, f1, g1, i2, j2, k2, f2, g2, i3, j3, k3, f3, g3);
          for (int c = 0; c < 8; c++) printf(" %d", cls[c] ? __builtin_ctz(cls[c]) : -1);
          printf("\n");
          if (want_t4) t4(1); else t3(1);
          fflush(stdout);
          if (nfound > 5) { printf("enough\n"); return 0; }
        }
      }
    }
  }
  printf("encodings %ld tried %ld found %ld\n", nenc, ntried, nfound);
}

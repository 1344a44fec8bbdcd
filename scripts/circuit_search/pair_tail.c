// Exhaustive search: does a T-gate (3-input LUT) circuit compute the B3/S23
// next state from a shared 3-plane pair-sum P (binary) + a 2-bit row sum X + alive c?
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef uint64_t u64;
static u64 IN[6], CARE, TGT;
static u64 gate(u64 a, u64 b, u64 c, int f) {
  u64 r = 0;
  for (int m = 0; m < 8; m++) if (f >> m & 1) {
    u64 t = ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
    r |= t;
  }
  return r;
}
static int func_of(const u64* s, int k) {
  // target is a function of signals s[0..k) on care rows
  u64 stack[64]; int n = 1; stack[0] = CARE;
  for (int i = 0; i < k; i++) {
    int nn = 0; u64 tmp[64];
    for (int j = 0; j < n; j++) {
      u64 a = stack[j] & s[i], b = stack[j] & ~s[i];
      if (a && (a & TGT) && (a & ~TGT)) tmp[nn++] = a;
      if (b && (b & TGT) && (b & ~TGT)) tmp[nn++] = b;
    }
    n = nn; memcpy(stack, tmp, n * sizeof(u64));
    if (!n) return 1;
  }
  return n == 0;
}
static u64 canon(u64 t) { u64 a = t & CARE, b = ~t & CARE; return a < b ? a : b; }
int main(int argc, char** argv) {
  // rows: bit0..2 = P, bit3..4 = X, bit5 = c
  for (int r = 0; r < 64; r++) {
    int P = r & 7, X = (r >> 3) & 3, c = (r >> 5) & 1;
    for (int i = 0; i < 6; i++) if (r >> i & 1) IN[i] |= 1ull << r;
    int care = P <= 6 && !(c && P == 0);
    if (care) CARE |= 1ull << r;
    int S = P + X;
    if (S == 3 || (S == 4 && c)) TGT |= 1ull << r;
  }
  // g1 candidates
  static u64 G1[6000]; int n1 = 0;
  for (int i = 0; i < 6; i++) for (int j = i + 1; j < 6; j++) for (int k = j + 1; k < 6; k++)
    for (int f = 0; f < 256; f++) {
      u64 t = gate(IN[i], IN[j], IN[k], f), c = canon(t);
      if (!c) continue;
      int dup = 0;
      for (int q = 0; q < 6 && !dup; q++) dup = canon(IN[q]) == c;
      for (int q = 0; q < n1 && !dup; q++) dup = canon(G1[q]) == c;
      if (!dup) G1[n1++] = t;
    }
  printf("g1 candidates %d\n", n1);
  long hits3 = 0, hits4 = 0;
#pragma omp parallel for schedule(dynamic) reduction(+:hits3,hits4)
  for (int a = 0; a < n1; a++) {
    u64 sig[8]; memcpy(sig, IN, sizeof IN); sig[6] = G1[a];
    for (int i = 0; i < 7; i++) for (int j = i + 1; j < 7; j++) for (int k = j + 1; k < 7; k++)
      for (int f = 0; f < 256; f++) {
        u64 t = gate(sig[i], sig[j], sig[k], f), c = canon(t);
        if (!c) continue;
        int dup = 0;
        for (int q = 0; q < 7 && !dup; q++) dup = canon(sig[q]) == c;
        if (dup) continue;
        sig[7] = t;
        // T=3: final over a triple containing g2
        for (int x = 0; x < 7; x++) for (int y = x + 1; y < 7; y++) {
          u64 s3[3] = {sig[x], sig[y], t};
          if (func_of(s3, 3)) {
            hits3++;
#pragma omp critical
            if (hits3 < 5) printf("T3: g1=%016llx g2=(%d,%d,%d,%02x) final(%d,%d,g2)\n", (unsigned long long)G1[a], i, j, k, f, x, y);
          }
        }
        // T=4 necessary: target function of 5 signals incl g2
        for (int x = 0; x < 7; x++) for (int y = x + 1; y < 7; y++) for (int z = y + 1; z < 7; z++) for (int w = z + 1; w < 7; w++) {
          u64 s5[5] = {t, sig[x], sig[y], sig[z], sig[w]};
          if (!func_of(s5, 5)) continue;
          // exact: choose 3 of the 5 for g3, 2 for the final gate's others
          int idx[5] = {0, 1, 2, 3, 4};
          for (int m = 0; m < 32; m++) {
            if (__builtin_popcount(m) != 3) continue;
            u64 s[3], yz[2]; int ns = 0, ny = 0;
            for (int b = 0; b < 5; b++) if (m >> b & 1) s[ns++] = s5[idx[b]]; else yz[ny++] = s5[idx[b]];
            for (int flips = 0; flips < 16; flips++) {
              int need[8]; for (int q = 0; q < 8; q++) need[q] = -1;
              int ok = 1;
              for (int r = 0; r < 64 && ok; r++) {
                if (!(CARE >> r & 1)) continue;
                int cls = (int)(yz[0] >> r & 1) | (int)(yz[1] >> r & 1) << 1;
                // is class constant?
                u64 cm = CARE & ((cls & 1) ? yz[0] : ~yz[0]) & ((cls & 2) ? yz[1] : ~yz[1]);
                if (!(cm & TGT) || !(cm & ~TGT)) continue;
                int pat = (int)(s[0] >> r & 1) << 2 | (int)(s[1] >> r & 1) << 1 | (int)(s[2] >> r & 1);
                int v = (int)(TGT >> r & 1) ^ (flips >> cls & 1);
                if (need[pat] < 0) need[pat] = v; else if (need[pat] != v) ok = 0;
              }
              if (ok) {
                hits4++;
#pragma omp critical
                if (hits4 < 20) printf("T4: g1=%016llx g2=(%d,%d,%d,%02x) subset=(%d,%d,%d,%d) m=%x flips=%x\n", (unsigned long long)G1[a], i, j, k, f, x, y, z, w, m, flips);
                goto next5;
              }
            }
          }
        next5:;
        }
      }
  }
  printf("hits3=%ld hits4=%ld\n", hits3, hits4);
}

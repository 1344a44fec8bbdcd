// All injective 6-class -> 3-bit codes (mod plane permutation/complement): is there a T=3 tail?
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef uint64_t u64;
static u64 gate64(u64 a, u64 b, u64 c, int f) {
  u64 r = 0;
  for (int m = 0; m < 8; m++) if (f >> m & 1) r |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
  return r;
}
static int func_of(u64 CARE, u64 TGT, const u64* s, int k) {
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
int main() {
  int perm[6][3] = {{0,1,2},{0,2,1},{1,0,2},{1,2,0},{2,0,1},{2,1,0}};
  static int codes[30000][6]; int nc = 0;
  static unsigned char seen[1 << 18];
  int c[6];
  for (c[0] = 0; c[0] < 8; c[0]++) for (c[1] = 0; c[1] < 8; c[1]++) for (c[2] = 0; c[2] < 8; c[2]++)
  for (c[3] = 0; c[3] < 8; c[3]++) for (c[4] = 0; c[4] < 8; c[4]++) for (c[5] = 0; c[5] < 8; c[5]++) {
    int used = 0, ok = 1;
    for (int i = 0; i < 6; i++) { if (used >> c[i] & 1) ok = 0; used |= 1 << c[i]; }
    if (!ok) continue;
    unsigned best = ~0u;
    for (int p = 0; p < 6; p++) for (int fl = 0; fl < 8; fl++) {
      unsigned key = 0;
      for (int i = 0; i < 6; i++) {
        int b[3] = {c[i] & 1, c[i] >> 1 & 1, c[i] >> 2 & 1}, n = 0;
        for (int q = 0; q < 3; q++) n |= (b[perm[p][q]] ^ (fl >> q & 1)) << q;
        key |= (unsigned)n << (3 * i);
      }
      if (key < best) best = key;
    }
    if (seen[best]) continue;
    seen[best] = 1;
    for (int i = 0; i < 6; i++) codes[nc][i] = best >> (3 * i) & 7;
    nc++;
  }
  printf("codes %d\n", nc);
  int hits = 0;
#pragma omp parallel for schedule(dynamic) reduction(+:hits)
  for (int e = 0; e < nc; e++) {
    u64 IN[6] = {0}, CARE = 0, TGT = 0;
    int cls_of_code[8]; for (int q = 0; q < 8; q++) cls_of_code[q] = -1;
    for (int i = 0; i < 6; i++) cls_of_code[codes[e][i]] = i;
    for (int r = 0; r < 64; r++) {
      for (int i = 0; i < 6; i++) if (r >> i & 1) IN[i] |= 1ull << r;
      int code = r & 7, X = r >> 3 & 3, cc = r >> 5 & 1, s = cls_of_code[code];
      if (s < 0 || (cc && s == 0)) continue;
      CARE |= 1ull << r;
      int S = s + X;
      if (S == 3 || (S == 4 && cc)) TGT |= 1ull << r;
    }
    int found = 0;
    for (int i = 0; i < 6 && !found; i++) for (int j = i + 1; j < 6 && !found; j++) for (int k = j + 1; k < 6 && !found; k++)
    for (int f = 0; f < 256 && !found; f++) {
      u64 sig[8]; memcpy(sig, IN, sizeof IN); sig[6] = gate64(IN[i], IN[j], IN[k], f);
      for (int i2 = 0; i2 < 7 && !found; i2++) for (int j2 = i2 + 1; j2 < 7 && !found; j2++) for (int k2 = j2 + 1; k2 < 7 && !found; k2++) {
        if (k2 != 6 && 0) continue;
        for (int f2 = 0; f2 < 256 && !found; f2++) {
          u64 t = gate64(sig[i2], sig[j2], sig[k2], f2);
          for (int x = 0; x < 7 && !found; x++) for (int y = x + 1; y < 7 && !found; y++) {
            u64 s3[3] = {sig[x], sig[y], t};
            if (func_of(CARE, TGT, s3, 3)) {
              found = 1;
#pragma omp critical
              printf("code %d%d%d%d%d%d: g1=(%d%d%d,%02x) g2=(%d%d%d,%02x) fin(%d,%d,g2)\n", codes[e][0], codes[e][1], codes[e][2], codes[e][3], codes[e][4], codes[e][5], i, j, k, f, i2, j2, k2, f2, x, y);
            }
          }
        }
      }
    }
    hits += found;
  }
  printf("hits %d\n", hits);
}

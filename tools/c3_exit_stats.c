// Offline analysis (CPU, not part of the product): input = out-CSR dump (u64 V, u64 E, u64 rp[V+1], u32 col[E])
// written from orientdb_amd.graph.rmat_csr(24); output = per-level in-edges a pull reads with and without the early exit.
// build: gcc -O2 -o /tmp/c3_exit_stats tools/c3_exit_stats.c
// For C3 (64-root MS-BFS, 4 levels over out-edges): per level, in-edges a bottom-up pull scans in full
// vs with a per-vertex early exit once the OR of gathered masks covers the vertex's needed lanes
// (in-lists hub-first by source out-degree, as k_bfs_pull's annotated col).
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb"); uint64_t V, E; fread(&V, 8, 1, f); fread(&E, 8, 1, f);
  uint64_t *rp = malloc((V + 1) * 8); uint32_t *col = malloc(E * 4);
  fread(rp, 8, V + 1, f); fread(col, 4, E, f); fclose(f);
  // sources in descending out-degree (counting sort by degree)
  uint64_t maxd = 0; for (uint64_t v = 0; v < V; ++v) { uint64_t d = rp[v+1]-rp[v]; if (d > maxd) maxd = d; }
  uint64_t *cnt = calloc(maxd + 2, 8);
  for (uint64_t v = 0; v < V; ++v) cnt[rp[v+1]-rp[v]]++;
  uint64_t acc = 0; for (int64_t d = maxd; d >= 0; --d) { uint64_t c = cnt[d]; cnt[d] = acc; acc += c; }
  uint32_t *order = malloc(V * 4); for (uint64_t v = 0; v < V; ++v) order[cnt[rp[v+1]-rp[v]]++] = (uint32_t)v;
  uint64_t *irp = calloc(V + 1, 8); for (uint64_t e = 0; e < E; ++e) irp[col[e] + 1]++;
  for (uint64_t v = 0; v < V; ++v) irp[v+1] += irp[v];
  uint64_t *pos = malloc(V * 8); memcpy(pos, irp, V * 8);
  uint32_t *icol = malloc(E * 4);
  for (uint64_t i = 0; i < V; ++i) { uint32_t u = order[i]; for (uint64_t e = rp[u]; e < rp[u+1]; ++e) icol[pos[col[e]]++] = u; }
  uint64_t *vis = calloc(V, 8), *fr = calloc(V, 8), *nx = calloc(V, 8);
  for (int i = 0; i < 64; ++i) { vis[i] |= 1ull << i; fr[i] |= 1ull << i; }
  for (int lvl = 1; lvl <= 4; ++lvl) {
    uint64_t live = 0, nfr = 0; for (uint64_t v = 0; v < V; ++v) { live |= fr[v]; nfr += fr[v] != 0; }
    uint64_t full = 0, ex = 0, nv = 0, ex1 = 0, ex4 = 0, ex16 = 0, hist_full_nv = 0;
    for (uint64_t v = 0; v < V; ++v) {
      uint64_t need = live & ~vis[v]; nx[v] = 0;
      if (!need || irp[v+1] == irp[v]) continue;
      nv++; uint64_t deg = irp[v+1]-irp[v]; full += deg;
      uint64_t o = 0, k = 0;
      for (uint64_t e = irp[v]; e < irp[v+1]; ++e) { o |= fr[icol[e]]; ++k; if ((o & need) == need) break; }
      if ((o & need) == need) { if (k <= 1) ex1++; if (k <= 4) ex4++; if (k <= 16) ex16++; } else hist_full_nv++;
      ex += k; nx[v] = o & need;
    }
    uint64_t nd = 0; for (uint64_t v = 0; v < V; ++v) { vis[v] |= nx[v]; fr[v] = nx[v]; nd += nx[v] != 0; }
    printf("level %d: frontier %llu vertices, live lanes %d; pull rows %llu; in-edges full %llu, early-exit %llu (%.1f%%); covered within 1/4/16 edges: %llu/%llu/%llu, never covered %llu; next frontier %llu\n",
           lvl, (unsigned long long)nfr, __builtin_popcountll(live), (unsigned long long)nv, (unsigned long long)full,
           (unsigned long long)ex, 100.0 * ex / (full ? full : 1), (unsigned long long)ex1, (unsigned long long)ex4,
           (unsigned long long)ex16, (unsigned long long)hist_full_nv, (unsigned long long)nd);
    fflush(stdout);
  }
  return 0;
}

// Offline analysis (CPU, not part of the product): input = out-CSR dump (u64 V, u64 E, u64 rp[V+1],
// u32 col[E]) written from orientdb_amd.graph.rmat_csr(24). For C3 (64-root MS-BFS over out-edges), per
// level: the in-edges a bottom-up pull reads, split by the source's out-degree rank (the pull kernel's
// LDS hubs, the packed hub array, the rest) and by whether the source is in the frontier — what a probe
// filter in LDS would keep away from L2.
// build: gcc -O2 -o /tmp/c3_sparse_stats tools/c3_sparse_stats.c
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  uint64_t V, E;
  if (fread(&V, 8, 1, f) != 1 || fread(&E, 8, 1, f) != 1) return 1;
  uint64_t *rp = malloc((V + 1) * 8);
  uint32_t *col = malloc(E * 4);
  if (fread(rp, 8, V + 1, f) != V + 1 || fread(col, 4, E, f) != E) return 1;
  fclose(f);
  const uint64_t lds_hubs = argc > 2 ? strtoull(argv[2], 0, 10) : 11500, hubs = argc > 3 ? strtoull(argv[3], 0, 10) : 1u << 20;
  // out-degree rank of every vertex (counting sort, descending)
  uint64_t maxd = 0;
  for (uint64_t v = 0; v < V; ++v) if (rp[v + 1] - rp[v] > maxd) maxd = rp[v + 1] - rp[v];
  uint64_t *cnt = calloc(maxd + 2, 8);
  for (uint64_t v = 0; v < V; ++v) cnt[rp[v + 1] - rp[v]]++;
  uint64_t acc = 0;
  for (int64_t d = maxd; d >= 0; --d) { uint64_t c = cnt[d]; cnt[d] = acc; acc += c; }
  uint32_t *rank = malloc(V * 4);
  for (uint64_t v = 0; v < V; ++v) rank[v] = (uint32_t)cnt[rp[v + 1] - rp[v]]++;
  uint64_t *irp = calloc(V + 1, 8);
  for (uint64_t e = 0; e < E; ++e) irp[col[e] + 1]++;
  for (uint64_t v = 0; v < V; ++v) irp[v + 1] += irp[v];
  uint64_t *pos = malloc(V * 8);
  memcpy(pos, irp, V * 8);
  uint32_t *icol = malloc(E * 4);
  for (uint64_t u = 0; u < V; ++u)
    for (uint64_t e = rp[u]; e < rp[u + 1]; ++e) icol[pos[col[e]]++] = (uint32_t)u;
  uint64_t *vis = calloc(V, 8), *fr = calloc(V, 8), *nx = calloc(V, 8);
  for (int i = 0; i < 64; ++i) { vis[i] |= 1ull << i; fr[i] |= 1ull << i; }
  for (int lvl = 1; lvl <= 4; ++lvl) {
    uint64_t live = 0, nfr = 0, pushE = 0;
    for (uint64_t v = 0; v < V; ++v) if (fr[v]) { live |= fr[v]; nfr++; pushE += rp[v + 1] - rp[v]; }
    // [class: 0 lds hub, 1 hub, 2 other][0 not in frontier, 1 in frontier, 2 useful (fr & need)]
    uint64_t c[3][3] = {{0}}, nv = 0, words_hit = 0;
    for (uint64_t v = 0; v < V; ++v) {
      const uint64_t need = live & ~vis[v];
      nx[v] = 0;
      if (!need || irp[v + 1] == irp[v]) continue;
      nv++;
      uint64_t o = 0;
      for (uint64_t e = irp[v]; e < irp[v + 1]; ++e) {
        const uint32_t u = icol[e];
        const int k = rank[u] < lds_hubs ? 0 : rank[u] < hubs ? 1 : 2;
        c[k][0]++;
        if (fr[u]) c[k][1]++;
        if (fr[u] & need) c[k][2]++;
        o |= fr[u];
      }
      nx[v] = o & need;
    }
    uint64_t nd = 0;
    for (uint64_t v = 0; v < V; ++v) { vis[v] |= nx[v]; fr[v] = nx[v]; nd += nx[v] != 0; }
    // frontier words of 64 vertices in id order and in rank order: how selective a coarse bitmap is
    uint64_t nw = (V + 63) / 64, wid = 0, wrk = 0;
    uint8_t *wi = calloc(nw, 1), *wr = calloc(nw, 1);
    for (uint64_t v = 0; v < V; ++v) if (fr[v]) { wi[v >> 6] = 1; wr[rank[v] >> 6] = 1; }
    for (uint64_t w = 0; w < nw; ++w) { wid += wi[w]; wrk += wr[w]; }
    free(wi); free(wr);
    (void)words_hit;
    printf("level %d: frontier %llu (push edges %llu), vertices needing lanes %llu, next frontier %llu; next-frontier 64-vertex words set: by id %llu, by rank %llu of %llu\n",
           lvl, (unsigned long long)nfr, (unsigned long long)pushE, (unsigned long long)nv, (unsigned long long)nd,
           (unsigned long long)wid, (unsigned long long)wrk, (unsigned long long)nw);
    const char *nm[3] = {"lds hubs", "hubs", "other"};
    for (int k = 0; k < 3; ++k)
      printf("   in-edges from %-8s %11llu  in frontier %11llu  useful %11llu\n", nm[k], (unsigned long long)c[k][0],
             (unsigned long long)c[k][1], (unsigned long long)c[k][2]);
  }
  return 0;
}

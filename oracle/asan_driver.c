/*
 * ORACLE self-check (test infrastructure only): drives every entry point of raster_cpu.c on
 * seeded random triangles — forward with and without the clipped-face neighbour rule, the pair
 * mode, a pixel window, K > 1 and blur, the backward and the projection — so that a build with
 * -fsanitize=address,undefined (oracle/Makefile target `asan`) checks the restatement for
 * out-of-bounds accesses and undefined behaviour. Exit status 0 = clean run.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_raster_fwd(const float*, const int64_t*, const int64_t*, int, int, int, int, float, int, int, int,
                    int64_t*, float*, float*, float*);
void orc_raster_fwd_ex(const float*, const int64_t*, const int64_t*, const int64_t*, int, int, int, int, float,
                       int, int, int, int, int, int, int, int64_t*, float*, float*, float*);
void orc_raster_fwd_pairs(const float*, const int64_t*, const int64_t*, const int64_t*, int, int, int, int, float,
                          int, int, int, int64_t*, float*, float*, float*);
void orc_raster_bwd(const float*, const int64_t*, const float*, const float*, const float*, int, int, int, int,
                    int, int, float*);
void orc_project_faces(const float*, const int32_t*, int64_t, const float*, int, float*);

static uint32_t rng = 12345u;
static float frand(void) { rng = rng * 1664525u + 1013904223u; return (float)(rng >> 8) / 16777216.0f; }

int main(void) {
  const int N = 2, F = 300, H = 24, W = 32, K = 4;
  float* fv = malloc(sizeof(float) * 9 * N * F);
  for (int i = 0; i < N * F; ++i) {
    const float cx = frand() * 2.4f - 1.2f, cy = frand() * 2.4f - 1.2f, z = 0.3f + 2.0f * frand();
    for (int c = 0; c < 3; ++c) {
      fv[9 * i + 3 * c] = cx + 0.3f * (frand() - 0.5f);
      fv[9 * i + 3 * c + 1] = cy + 0.3f * (frand() - 0.5f);
      fv[9 * i + 3 * c + 2] = z + 0.2f * (frand() - 0.5f);
    }
  }
  fv[9 * 5] = NAN; /* a non-finite face is skipped */
  int64_t first[2] = {0, F}, count[2] = {F, F};
  int64_t* nb = malloc(sizeof(int64_t) * N * F);
  for (int i = 0; i < N * F; ++i) nb[i] = -1;
  for (int i = 10; i + 1 < N * F; i += 37) { nb[i] = i + 1; nb[i + 1] = i; }
  const size_t P = (size_t)N * H * W * K;
  int64_t* p2f = malloc(sizeof(int64_t) * P);
  float *zb = malloc(sizeof(float) * P), *ba = malloc(sizeof(float) * 3 * P), *di = malloc(sizeof(float) * P);
  orc_raster_fwd(fv, first, count, N, H, W, 1, 0.0f, 1, 0, 0, p2f, zb, ba, di);
  orc_raster_fwd_ex(fv, first, count, nb, N, H, W, K, 1e-3f, 1, 1, 1, 3, 17, 5, 29, p2f, zb, ba, di);
  orc_raster_fwd_pairs(fv, first, count, nb, N, H, W, K, 1e-3f, 0, 1, 0, p2f, zb, ba, di);
  orc_raster_fwd_ex(fv, first, count, nb, N, H, W, K, 2e-4f, 1, 1, 0, 0, 0, 0, 0, p2f, zb, ba, di);
  float *gz = malloc(sizeof(float) * P), *gb = malloc(sizeof(float) * 3 * P), *gd = malloc(sizeof(float) * P);
  for (size_t i = 0; i < P; ++i) { gz[i] = frand(); gd[i] = frand(); gb[3 * i] = frand(); gb[3 * i + 1] = frand(); gb[3 * i + 2] = frand(); }
  float* gfv = calloc(9 * (size_t)N * F, sizeof(float));
  orc_raster_bwd(fv, p2f, gz, gb, gd, N, H, W, K, 1, 1, gfv);
  int covered = 0;
  for (size_t i = 0; i < P; ++i) covered += p2f[i] >= 0;
  const int V = 50;
  float* verts = malloc(sizeof(float) * 3 * V);
  for (int i = 0; i < 3 * V; ++i) verts[i] = frand() - 0.5f;
  int32_t faces[3 * 40];
  for (int i = 0; i < 3 * 40; ++i) faces[i] = (int32_t)(frand() * V) % V;
  float views[2 * 16] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 2, 1, 0, 1, 0, 0, 1, 0, 1, 0, 0, 0, 0, 1, 0.1f, 0.2f, 3, 1.5f, 0, 1.5f, 0};
  float* pfv = malloc(sizeof(float) * 9 * 2 * 40);
  orc_project_faces(verts, faces, 40, views, 2, pfv);
  printf("oracle asan driver ok: %d covered fragments\n", covered);
  free(fv); free(nb); free(p2f); free(zb); free(ba); free(di); free(gz); free(gb); free(gd); free(gfv);
  free(verts); free(pfv);
  return covered > 0 ? 0 : 1;
}

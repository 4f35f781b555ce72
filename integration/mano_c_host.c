/*
 * mano_c_host.c -- a plain-C host of the MI355X MANO forward (no Python, no
 * torch): what a C / C++ application links against instead of calling the
 * reference's numpy MANOModel.update() (mano_np.py:79-115) per hand.
 *
 *   mano_c_host <model.bin> <n_hands> <seed> <out.bin> [n_devices]
 *
 * model.bin: the dump_model.py arrays as float64, in the order and shapes
 * of mano_model_create (include/mano_hip.h): int32 V, then template [V][3],
 * shape basis [V][3][10], pose basis [V][3][135], J_regressor [16][V],
 * skinning weights [V][16], int32 parents [16], PCA basis [45][45], PCA mean
 * [45].  The program builds one model handle per device, generates hands
 * 0 .. n-1 of the counter-based synthetic batch (mano_synthetic_inputs, each
 * device its contiguous shard by global index), runs mano_forward on every
 * device from this one thread, assembles all verts + posed joints on device 0
 * with ONE RCCL group (mano_comm_create_all, mano_group_start, mano_gather per
 * device (each checked first with mano_gather_check), mano_group_end; ABI 7) and writes them to out.bin as float32
 * [n][V][3] then [n][16][3].  Exit status 0 on success; every failing call's
 * mano_last_error() on stderr.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mano_hip.h"

#define CHECK(call)                                                              \
  do {                                                                           \
    int rc_ = (call);                                                            \
    if (rc_ != MANO_OK) {                                                        \
      fprintf(stderr, "%s:%d: %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_,   \
              mano_last_error());                                                \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

static void* read_exact(FILE* f, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "model file truncated (%zu bytes wanted)\n", bytes);
    exit(2);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s model.bin n_hands seed out.bin [n_devices]\n", argv[0]);
    return 1;
  }
  const long long n_total = atoll(argv[2]);
  const unsigned long long seed = strtoull(argv[3], NULL, 10);
  const int n_dev = argc > 5 ? atoi(argv[5]) : 1;
  if (n_total < 1 || n_dev < 1 || n_dev > 64) {
    fprintf(stderr, "bad n_hands / n_devices\n");
    return 1;
  }
  if (mano_abi_version() < 7) {
    fprintf(stderr, "libmano_hip ABI %d < 7\n", mano_abi_version());
    return 2;
  }

  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 2;
  }
  int32_t V = 0;
  if (fread(&V, sizeof V, 1, f) != 1 || V < 32) {
    fprintf(stderr, "bad vertex count\n");
    return 2;
  }
  double* tmpl = read_exact(f, sizeof(double) * V * 3);
  double* sdirs = read_exact(f, sizeof(double) * V * 3 * MANO_N_SHAPE);
  double* pdirs = read_exact(f, sizeof(double) * V * 3 * MANO_N_POSE_FEATS);
  double* jreg = read_exact(f, sizeof(double) * MANO_N_JOINTS * V);
  double* wts = read_exact(f, sizeof(double) * V * MANO_N_JOINTS);
  int32_t* parents = read_exact(f, sizeof(int32_t) * MANO_N_JOINTS);
  double* pca = read_exact(f, sizeof(double) * MANO_N_PCA * MANO_N_PCA);
  double* pmean = read_exact(f, sizeof(double) * MANO_N_PCA);
  fclose(f);

  /* contiguous shards of the global batch, rank r on device r */
  long long* first = calloc(n_dev + 1, sizeof *first);
  const long long per = (n_total + n_dev - 1) / n_dev;
  for (int r = 0; r <= n_dev; ++r) first[r] = r * per < n_total ? r * per : n_total;

  mano_model** models = calloc(n_dev, sizeof *models);
  void **betas = calloc(n_dev, sizeof(void*)), **pose = calloc(n_dev, sizeof(void*));
  void **verts = calloc(n_dev, sizeof(void*)), **joints = calloc(n_dev, sizeof(void*));
  void** ws = calloc(n_dev, sizeof(void*));
  size_t* ws_bytes = calloc(n_dev, sizeof(size_t));
  size_t* vbytes = calloc(n_dev, sizeof(size_t));
  size_t* jbytes = calloc(n_dev, sizeof(size_t));
  int* devices = calloc(n_dev, sizeof(int));
  const size_t vrow = (size_t)V * 3 * sizeof(float), jrow = MANO_N_JOINTS * 3 * sizeof(float);
  void *all_v = NULL, *all_j = NULL;

  for (int r = 0; r < n_dev; ++r) {
    const long long n = first[r + 1] - first[r];
    devices[r] = r;
    vbytes[r] = (size_t)n * vrow;
    jbytes[r] = (size_t)n * jrow;
    CHECK(mano_model_create(r, V, tmpl, sdirs, pdirs, jreg, wts, parents, pca, pmean, &models[r]));
    CHECK(mano_alloc(r, (size_t)n * MANO_N_SHAPE * sizeof(float), &betas[r]));
    CHECK(mano_alloc(r, (size_t)n * MANO_N_JOINTS * 3 * sizeof(float), &pose[r]));
    ws_bytes[r] = mano_forward_workspace_bytes(models[r], n);
    CHECK(mano_alloc(r, ws_bytes[r], &ws[r]));
    if (r == 0) {
      /* the assembled outputs; device 0's own shard is computed in place */
      CHECK(mano_alloc(0, (size_t)n_total * vrow, &all_v));
      CHECK(mano_alloc(0, (size_t)n_total * jrow, &all_j));
      verts[0] = all_v;
      joints[0] = all_j;
    } else {
      CHECK(mano_alloc(r, vbytes[r], &verts[r]));
      CHECK(mano_alloc(r, jbytes[r], &joints[r]));
    }
  }
  /* every launch is asynchronous (null stream of each device): one thread
     keeps all devices busy */
  for (int r = 0; r < n_dev; ++r) {
    const long long n = first[r + 1] - first[r];
    if (n == 0) continue;
    CHECK(mano_synthetic_inputs(r, seed, first[r], n, 1.0f, 0.5f, 1.0f, (float*)betas[r],
                                (float*)pose[r], NULL, NULL));
    CHECK(mano_forward(models[r], n, betas[r], MANO_N_SHAPE, pose[r], NULL, verts[r], joints[r],
                       NULL, NULL, NULL, ws[r], ws_bytes[r], NULL));
  }
  /* one RCCL group from this thread: every shard to device 0 */
  mano_comm** comms = calloc(n_dev, sizeof *comms);
  CHECK(mano_comm_create_all(n_dev, devices, comms));
  /* every call of the group checked BEFORE the group posts anything (ABI 7):
     a call refused half way would leave a root receive without its send */
  for (int r = 0; r < n_dev; ++r) CHECK(mano_gather_check(comms[r], verts[r], vbytes[r], r == 0 ? all_v : NULL, vbytes, 0));
  for (int r = 0; r < n_dev; ++r) CHECK(mano_gather_check(comms[r], joints[r], jbytes[r], r == 0 ? all_j : NULL, jbytes, 0));
  CHECK(mano_group_start());
  for (int r = 0; r < n_dev; ++r) CHECK(mano_gather(comms[r], verts[r], vbytes[r], r == 0 ? all_v : NULL, vbytes, 0, NULL));
  for (int r = 0; r < n_dev; ++r) CHECK(mano_gather(comms[r], joints[r], jbytes[r], r == 0 ? all_j : NULL, jbytes, 0, NULL));
  CHECK(mano_group_end());
  for (int r = 0; r < n_dev; ++r) CHECK(mano_synchronize(r));
  for (int r = 0; r < n_dev; ++r) {
    int32_t st = 0;
    CHECK(mano_model_device_status(models[r], &st, MANO_STATUS_CLEAR));
    if (st) {
      fprintf(stderr, "device %d status 0x%x\n", r, st);
      return 3;
    }
  }

  float* hv = malloc((size_t)n_total * vrow);
  float* hj = malloc((size_t)n_total * jrow);
  CHECK(mano_memcpy(0, hv, all_v, (size_t)n_total * vrow, MANO_MEMCPY_DEVICE_TO_HOST, NULL));
  CHECK(mano_memcpy(0, hj, all_j, (size_t)n_total * jrow, MANO_MEMCPY_DEVICE_TO_HOST, NULL));
  FILE* o = fopen(argv[4], "wb");
  if (!o || fwrite(hv, 1, (size_t)n_total * vrow, o) != (size_t)n_total * vrow ||
      fwrite(hj, 1, (size_t)n_total * jrow, o) != (size_t)n_total * jrow) {
    perror(argv[4]);
    return 2;
  }
  fclose(o);

  for (int r = 0; r < n_dev; ++r) {
    CHECK(mano_comm_destroy(comms[r]));
    CHECK(mano_free(r, betas[r]));
    CHECK(mano_free(r, pose[r]));
    CHECK(mano_free(r, ws[r]));
    if (r > 0) {
      CHECK(mano_free(r, verts[r]));
      CHECK(mano_free(r, joints[r]));
    }
    CHECK(mano_model_destroy(models[r]));
  }
  CHECK(mano_free(0, all_v));
  CHECK(mano_free(0, all_j));
  printf("mano_c_host: %lld hands on %d device(s), verts[0][0] = %.7f %.7f %.7f\n", n_total, n_dev,
         hv[0], hv[1], hv[2]);
  return 0;
}

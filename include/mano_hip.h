/*
 * mano_hip.h -- C ABI of the MI355X (gfx950) MANO forward pass.
 *
 * The reference (reyuwei/MANO-Hand) has no FFI: its boundary is the Python
 * object `MANOModel` in /root/reference/mano_np.py.  Each entry point below
 * replaces a named piece of that object; the Python host layer
 * (mano-hand_amd/mano_amd/) binds them with ctypes and re-creates the
 * reference surface on top (see INTEGRATION.md for the binding stub).
 *
 * Conventions
 *   - Every function returns an int status: MANO_OK (0) or a negative
 *     MANO_E* code; mano_last_error() gives the message (thread-local).
 *     No C++ exception crosses this ABI.
 *   - Array arguments are plain pointers with the sizes stated.  Model arrays
 *     given to mano_model_create are HOST float64 (the dump_model.py layout);
 *     every pointer given to the forward / stage / helper calls is a DEVICE
 *     pointer owned by the caller, on the model's device.
 *   - Launches are asynchronous on `stream` (a hipStream_t; NULL = the
 *     device's null stream).  Nothing blocks except model create/destroy,
 *     mano_model_device_status, mano_synchronize and NULL-stream mano_memcpy.
 *   - A model handle is bound to one device.  Calls on one handle may come
 *     from several host threads only if they use distinct workspaces.
 *   - Layouts are the reference's, row-major float32:
 *       betas     [n][10]       (betas_stride = 10, or 0 for one shared vector)
 *       pose      [n][16][3]    axis-angle per joint, joint 0 = global rotation
 *       trans     [n][3]        (extension: the reference has no translation)
 *       verts     [n][V][3]     = MANOModel.verts        (mano_np.py:113-115)
 *       joints    [n][16][3]    posed joints = G[:, :3, 3] (mano_np.py:96-104)
 *       rest_verts[n][V][3]     = MANOModel.rest_verts   (mano_np.py:91-93)
 *       rest_joints[n][16][3]   = MANOModel.J            (mano_np.py:83)
 *       rot_mats  [n][16][3][3] = MANOModel.R            (mano_np.py:86)
 */
#ifndef MANO_HIP_H
#define MANO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MANO_OK 0
#define MANO_EINVAL (-1)   /* bad argument (null pointer, bad size, bad layout) */
#define MANO_EHIP (-2)     /* HIP runtime error (allocation, copy, launch)      */
#define MANO_ESMALL (-3)   /* workspace smaller than mano_workspace_bytes()     */
#define MANO_ESTATE (-4)   /* handle destroyed / wrong device                   */
#define MANO_ECOMM (-5)    /* RCCL unavailable or a collective failed           */
#define MANO_EDEVICE (-6)  /* an earlier launch on this model raised a MANO_DEVICE_* bit:
                              its outputs are not valid (mano_model_device_status) */

#define MANO_N_JOINTS 16
#define MANO_N_SHAPE 10
#define MANO_N_POSE_FEATS 135
#define MANO_N_PCA 45

/* Arithmetic of the blend GEMM and LBS transform blend (mano_model_set_precision):
 *  FP32   exact fp32 on v_mfma_f32_16x16x4_f32 (the default);
 *  F16X3  every fp32 operand split into hi + lo halves (22 significant bits),
 *         products hi.hi + hi.lo + lo.hi accumulated in fp32 on
 *         v_mfma_f32_16x16x32_f16 (16/3 x the fp32 MFMA rate).  Same error
 *         order as FP32 vs the float64 reference (~1e-7 m); needs |beta| and
 *         the pose features within f16 range and skinning transforms < 1000.
 *         Used for verts-only forwards and for mano_stage_skin; a
 *         mano_forward / mano_forward_pca / mano_stage_blend_skin call that
 *         requests rest_verts runs the FP32 kernel (the f16x3 kernel with a
 *         rest_verts output is not built: its vectorized form miscomputed
 *         under load for a reason never explained).
 *         mano_stage_blend is always FP32. */
#define MANO_PRECISION_FP32 0
#define MANO_PRECISION_F16X3 1

typedef struct mano_model mano_model; /* opaque, device-resident model buffer */

/* Upload a model and build its device buffer.
 * Replaces MANOModel.__init__'s array binding (mano_np.py:17-33) for the
 * dump_model.py layout (dump_model.py:8-18).  Host float64 inputs:
 *   mesh_template    [V][3] (V >= 32) mesh_shape_basis [V][3][10]
 *   mesh_pose_basis  [V][3][135]     J_regressor      [16][V] (dense)
 *   skinning_weights [V][16]         parents          [16] int32, -1 at root,
 *                                                     parents[i] < i
 *   pose_pca_basis   [45][45]        pose_pca_mean    [45]   (both nullable)
 * The joint regression is folded in float64 here (J = Jreg.T + (Jreg.S) beta),
 * then everything is stored as float32 in MFMA-ready layouts. */
int mano_model_create(int device, int32_t n_verts,
                      const double* mesh_template, const double* mesh_shape_basis,
                      const double* mesh_pose_basis, const double* j_regressor,
                      const double* skinning_weights, const int32_t* parents,
                      const double* pose_pca_basis, const double* pose_pca_mean,
                      mano_model** out);

/* Select the arithmetic of mano_forward, mano_stage_blend_skin and
 * mano_stage_skin on this handle (MANO_PRECISION_*; default FP32).  Not
 * synchronised with launches already queued (they keep the mode they were
 * issued with). */
int mano_model_set_precision(mano_model* model, int32_t precision);
int mano_model_get_precision(const mano_model* model, int32_t* precision);

/* Free the device buffer.  NULL is accepted. */
int mano_model_destroy(mano_model* model);

/* Vertex count and device of a model. */
int mano_model_info(const mano_model* model, int32_t* n_verts, int32_t* device);

/* Device status of a model: the MANO_DEVICE_* bits kernels raised since the
 * last clear.  A set bit means some launch's outputs are not valid:
 *   MANO_DEVICE_SKIN_HANDOFF_TIMEOUT  the standalone LBS (mano_stage_skin) lost
 *     a hand-over between its memory and compute waves (a bounded LDS wait
 *     gave up -- reachable only through a broken protocol: the waves of a
 *     workgroup are co-resident); the verts of the units it could not
 *     confirm were not written.
 * Contract: launches are asynchronous, so the call that issued such a launch
 * has already returned MANO_OK; from the moment the bit is raised, EVERY
 * launching call on the model (mano_forward*, mano_stage_*,
 * mano_pose_from_pca) returns MANO_EDEVICE without launching, until this
 * function is called with MANO_STATUS_CLEAR.  The bits are flags in pinned
 * host memory that the kernels set with plain stores: this call waits for
 * every launch on the model's device (hipDeviceSynchronize; not with
 * MANO_STATUS_NO_WAIT, which reads what has landed so far), ORs them into
 * *status and, with MANO_STATUS_CLEAR, takes each with one host atomic
 * exchange -- concurrent callers never lose a bit, each reports it once. */
#define MANO_DEVICE_SKIN_HANDOFF_TIMEOUT 1
#define MANO_STATUS_CLEAR 1
#define MANO_STATUS_NO_WAIT 2
int mano_model_device_status(const mano_model* model, int32_t* status, int32_t flags);

/* Device workspace (bytes) for n_hands: `mano_workspace_bytes` covers every
 * call (the unfused stages keep v_posed in it); `mano_forward_workspace_bytes`
 * only what mano_forward / articulate / blend_skin use (X rows + transforms,
 * 1,408 B per hand). */
size_t mano_workspace_bytes(const mano_model* model, int64_t n_hands);
size_t mano_forward_workspace_bytes(const mano_model* model, int64_t n_hands);

/* Byte offsets of the intermediates inside the workspace (for inspection):
 * the blend-GEMM A operand rows X [n][160] = [beta | R - I features | 1 | 0..]
 * stored k-permuted (element k at 16(k>>4) + 4(k&3) + ((k>>2)&3)), the
 * skinning transforms [n][16][3][4], v_posed [n][V][3]. */
int mano_workspace_offsets(const mano_model* model, int64_t n_hands,
                           size_t* features_off, size_t* transforms_off,
                           size_t* vposed_off);

/* The full forward pass: MANOModel.update() (mano_np.py:79-115) for n_hands
 * independent hands = articulate + blend_skin (two launches).  verts is
 * required; joints, rest_verts, rest_joints, rot_mats and trans are nullable;
 * betas_stride 0 shares one beta row.  v_posed never touches HBM unless
 * rest_verts is requested. */
int mano_forward(const mano_model* model, int64_t n_hands,
                 const float* betas, int64_t betas_stride, const float* pose,
                 const float* trans, float* verts, float* joints,
                 float* rest_verts, float* rest_joints, float* rot_mats,
                 void* workspace, size_t workspace_bytes, void* stream);

/* The forward pass as separate kernels, callable one at a time (workspace of
 * mano_workspace_bytes), so each can be timed and its intermediates checked.
 * blend, skin and blend_skin read the X rows and transforms that the last
 * articulate (or mano_forward) on the same n_hands left in the same
 * workspace; the offsets depend on n_hands only (mano_workspace_offsets).
 *  articulate: Rodrigues (mano_np.py:117-148) + joint regression (:83) +
 *              pose features (:87-91) + kinematic chain (:96-104) +
 *              rest-pose removal (:106-110).
 *  blend:      v_posed = T + S.beta + P.features (:81, :87-93) on MFMA.
 *  skin:       LBS (:112-115), + trans.  rest_verts (NULL = the workspace's
 *              v_posed) may be verts itself: the LBS then runs in place
 *              (ABI 7; the blend writes v_posed into verts, the LBS
 *              overwrites it -- no second buffer, and its writes land on the
 *              blend's still-cached lines); any other overlap of the two is
 *              MANO_EINVAL. */
int mano_stage_articulate(const mano_model* model, int64_t n_hands,
                          const float* betas, int64_t betas_stride,
                          const float* pose, const float* trans, float* joints,
                          float* rest_joints, float* rot_mats, void* workspace,
                          size_t workspace_bytes, void* stream);
int mano_stage_blend(const mano_model* model, int64_t n_hands, float* rest_verts,
                     void* workspace, size_t workspace_bytes, void* stream);
int mano_stage_skin(const mano_model* model, int64_t n_hands,
                    const float* rest_verts, const float* trans, float* verts,
                    void* workspace, size_t workspace_bytes, void* stream);
/*  blend_skin: blend + skin fused (the LBS runs in the GEMM epilogue, v_posed
 *              stays on chip; written to rest_verts only when non-NULL). */
int mano_stage_blend_skin(const mano_model* model, int64_t n_hands, float* rest_verts,
                          const float* trans, float* verts, void* workspace,
                          size_t workspace_bytes, void* stream);

/* set_params' PCA branch (mano_np.py:66-72) on device:
 *   pose[h] = [ rot[h] | pca[h][:n_comps] . pose_pca_basis[:n_comps] + mean ]
 * pca [n][pca_stride] (stride 0 = shared), rot [n][3] (rot_stride 0 = shared). */
int mano_pose_from_pca(const mano_model* model, int64_t n_hands, const float* pca,
                       int32_t n_comps, int64_t pca_stride, const float* rot,
                       int64_t rot_stride, float* pose, void* stream);

/* set_params(pose_pca=..., global_rot=..., shape=...) (mano_np.py:48-77) for a
 * batch: the PCA map of mano_pose_from_pca runs as the prologue of the
 * articulation kernel (no pose round trip through HBM), then the forward
 * pass of mano_forward.  pca [n][pca_stride] (stride 0 = one shared row,
 * 0 <= n_comps <= 45; n_comps 0 gives the PCA mean), rot [n][3] (rot_stride 0
 * = shared; NULL = zero root rotation, the reference's initial `rot`).
 * pose_out (nullable) receives the [n][16][3] pose the kernels used -- bit for
 * bit what mano_pose_from_pca returns.  Needs a model created with the PCA
 * arrays.  Other arguments as mano_forward. */
int mano_forward_pca(const mano_model* model, int64_t n_hands, const float* betas,
                     int64_t betas_stride, const float* pca, int32_t n_comps,
                     int64_t pca_stride, const float* rot, int64_t rot_stride,
                     const float* trans, float* verts, float* joints, float* pose_out,
                     float* rest_verts, float* rest_joints, float* rot_mats,
                     void* workspace, size_t workspace_bytes, void* stream);

/* MANOModel.rodrigues (mano_np.py:117-148): n axis-angle vectors [n][3] ->
 * rotation matrices [n][3][3]. */
int mano_rodrigues(int device, int64_t n, const float* axis_angle, float* rot,
                   void* stream);

/* ---- Device memory and streams without a framework --------------------
 * So that the reference's own process (numpy + ctypes, no torch) can hold
 * the device buffers mano_forward reads and writes.
 * mano_alloc returns 256-byte aligned device memory on `device`;
 * mano_memcpy copies `bytes` in direction `kind` (MANO_MEMCPY_*), on
 * `stream` asynchronously, or synchronously when stream is NULL;
 * mano_synchronize waits for every launch on `device`. */
#define MANO_MEMCPY_HOST_TO_DEVICE 1
#define MANO_MEMCPY_DEVICE_TO_HOST 2
#define MANO_MEMCPY_DEVICE_TO_DEVICE 3
int mano_alloc(int device, size_t bytes, void** out);
int mano_free(int device, void* ptr);
int mano_memcpy(int device, void* dst, const void* src, size_t bytes, int32_t kind,
                void* stream);
int mano_synchronize(int device);
/* Pinned host memory mapped into every device's address space at the same
 * address (hipHostMalloc): mano_forward and the stage calls may take it as
 * their inputs and outputs directly -- the kernels read and write it over
 * the host link, no copy -- which for a batch-1 call is faster than a copy
 * each way (ABI 5).  Results are in host memory once the
 * launch's stream (or mano_synchronize) has completed. */
int mano_host_alloc(size_t bytes, void** out);
int mano_host_free(void* ptr);

/* ---- Synthetic workload (benchmarks, shard-invariance tests) ------------
 * Hand i of the batch is global hand first_index + i; its values are drawn
 * by Philox-4x32-10 keyed by `seed` with counter (global index, block), so a
 * shard [a, b) of a global batch reproduces exactly hands a..b-1 of the
 * 1-GPU batch.  Per hand, 16 Philox blocks give
 * 64 uint32 words w[0..63]: w[0..57] become 58 normals by Box-Muller on the
 * pairs (w[2m], w[2m+1]) (cos for the even member, sin for the odd),
 * betas [n][10] = beta_sigma * N[0..9], pose [n][16][3] = pose_sigma *
 * N[10..57], trans [n][3] = trans_range * (2 u(w[58..60]) - 1), with
 * u(w) = ((w >> 8) + 0.5) / 2^24 in (0, 1) and N = sqrt(-2 ln u(w[2m])) *
 * (cos, sin)(2 pi u(w[2m+1])), evaluated in float32.  Each output is
 * nullable. */
int mano_synthetic_inputs(int device, uint64_t seed, int64_t first_index, int64_t n_hands,
                          float beta_sigma, float pose_sigma, float trans_range,
                          float* betas, float* pose, float* trans, void* stream);

/* ---- Gather of per-rank shards to one GPU (RCCL over xGMI) --------------
 * The forward has no collective (hands are independent); this assembles the
 * shards of a data-parallel batch on `root` when the caller wants every
 * vertex on one device (BASELINE config C4).  One rank per GPU and process;
 * rank 0 makes the id with mano_comm_unique_id and hands it to the others
 * out of band.  mano_gather is a grouped RCCL send/recv: every peer sends
 * its `send_bytes` straight to root over its own xGMI link (no ring), root
 * lands rank r's bytes at recv + sum(rank_bytes[0..r-1]) (rank_bytes: the
 * per-rank sizes, read on root only; NULL = every rank sends send_bytes), so
 * ragged contiguous shards need no padding.  recv is read on root only.
 * The root may produce its own shard in place (send == recv + its offset):
 * then nothing is copied for it.  Asynchronous on `stream`.  RCCL
 * (librccl.so.1) is loaded on first use. */
#define MANO_COMM_ID_BYTES 128
typedef struct mano_comm mano_comm;
int mano_comm_unique_id(unsigned char* id /* [MANO_COMM_ID_BYTES] */);
int mano_comm_create(int device, int32_t n_ranks, int32_t rank, const unsigned char* id,
                     mano_comm** out);
int mano_comm_destroy(mano_comm* comm);
int mano_gather(mano_comm* comm, const void* send, size_t send_bytes, void* recv,
                const size_t* rank_bytes, int32_t root, void* stream);
/* Single-process form (ABI 6): ONE host thread drives n devices, as the
 * reference's own single-process batch loop would (data_explore.py:12-15;
 * ncclCommInitAll).  mano_comm_create_all makes one
 * communicator per device in one call (rank i on devices[i], distinct
 * devices; comms[n] out).  Calls on several of them from one thread go
 * between mano_group_start and mano_group_end (ncclGroupStart / End), which
 * issues them together: mano_gather on every comm with its own send buffer
 * and stream (recv on the root's) gathers all devices' shards onto the root
 * without any other thread or process.  Each comm is destroyed on its own. */
int mano_comm_create_all(int32_t n, const int* devices, mano_comm** comms);
int mano_group_start(void);
int mano_group_end(void);
/* Argument checks of one mano_gather call, without posting anything (ABI 7).
 * A mano_gather that fails its checks posts nothing, but inside a group the
 * calls BEFORE it have already posted theirs: ncclGroupEnd would launch a
 * half-built group (a root receive with no matching send never completes),
 * and RCCL has no way to abandon a group.  So a host that issues several
 * gathers in one group checks every one of them with mano_gather_check
 * first and calls mano_group_start only when all pass;
 * mano_gather runs exactly these checks, so a call that passes here is not
 * refused there.  (A HIP or RCCL failure after the checks -- a lost device --
 * still leaves the group's streams undefined.) */
int mano_gather_check(const mano_comm* comm, const void* send, size_t send_bytes,
                      const void* recv, const size_t* rank_bytes, int32_t root);
/* Size, rank and device of a communicator (each output nullable; ABI 7). */
int mano_comm_info(const mano_comm* comm, int32_t* n_ranks, int32_t* rank, int32_t* device);
/* Every rank receives every shard: RCCL's ring ncclAllGather of equal
 * `send_bytes` shards, rank r's bytes at recv + r * send_bytes on EVERY rank
 * (recv holds n_ranks * send_bytes; in place when send == recv + rank *
 * send_bytes, as RCCL allows).  The comparison form for mano_gather
 * (a ring is bound by one link per hop), and the call for
 * callers that want the whole batch on every device.  Asynchronous on
 * `stream`. */
int mano_allgather(mano_comm* comm, const void* send, size_t send_bytes, void* recv,
                   void* stream);

/* Message of the last failed call on this thread ("" if none). */
const char* mano_last_error(void);

/* ABI version, bumped on any signature change (4: + mano_allgather; 5: +
 * mano_host_alloc / mano_host_free; 6: + mano_comm_create_all /
 * mano_group_start / mano_group_end, MANO_EDEVICE, mano_model_device_status
 * flags; 7: + mano_gather_check / mano_comm_info, in-place mano_stage_skin). */
int mano_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MANO_HIP_H */

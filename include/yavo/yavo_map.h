/* yavo_map.h -- the shared map: keyframes and landmarks of a frame chunk packed into one
 * fixed-size device block per rank, exchanged between ranks by an all-gather (RCCL over xGMI), then placed in world
 * coordinates identically on every rank.
 *
 * Replaces the reference's Map::insertKeyFrame / Map::insertMapPoint (src/Map.cc:9-40; Map::LandMarksType keyed by
 * MapPoint::ptID, Map::FramesType keyed by Frame::frameID, include/Map.hpp:12-13) for a sharded sequence: the
 * reference's map is one process-wide object behind a mutex; here every rank builds the block of its own frame
 * chunk on the device and the all-gather hands each rank every block.
 *
 * Poses: the batch's tracks give rel_k = T_{k-1,k} (frame k-1's camera from frame k's, yv_batch_track). A block
 * holds L_k = rel_0 * rel_1 * ... * rel_k (Sophus products, left fold) for its keyframes and C = L_{n-1} in its
 * header, so with the anchor A = T_wc of the frame before the chunk, T_wc(k) = A * L_k. Placement runs the anchors
 * serially over the ranks (A_0 = base, A_{r+1} = A_r * C_r, base <- A_world) and rewrites every block in place:
 * keyframe T_wc = A_r * L_k, landmark X_w = T_wc(k) * X (X = the stereo-triangulated point in frame k's left
 * camera). Poses are Sophus SE3d::data() = {qx, qy, qz, qw, tx, ty, tz}. */
#ifndef YAVO_MAP_H
#define YAVO_MAP_H
#include <stdint.h>

#include "yavo.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct yv_map_header {
    double chunk[7];     /* C = L_{n-1}: the chunk's composed relative pose */
    int64_t first_frame; /* global index of the chunk's first frame */
    int32_t n_frames;    /* frames in the chunk */
    int32_t n_kf;        /* keyframes written */
    int32_t kf_every;    /* keyframe policy: global index % kf_every == 0 */
    int32_t lm_stride;   /* landmark slots per keyframe */
    int32_t max_kf;
    int32_t placed;      /* 0: block-local (L_k, camera X); 1: world (T_wc, X_w); 2: a sequence shard's export
                          * (yv_ba_window_export_block: the shard's own T_wc and X_w, relative to its first frame);
                          * 3: such an export placed in world coordinates */
    double pad[5];
} yv_map_header; /* 128 B */

typedef struct yv_keyframe {
    int64_t frame_id;    /* Frame::frameID: the global frame index */
    double T[7];         /* L_k before placement, T_wc after */
    int32_t n_landmarks; /* inlier landmarks written for this keyframe */
    int32_t pad;
} yv_keyframe; /* 72 B */

typedef struct yv_landmark {
    int64_t id;  /* MapPoint::ptID: frame_id << 16 | edge index */
    double X[3]; /* camera (frame_id's left camera) before placement, world after */
} yv_landmark; /* 32 B */

/* Bytes of one block: header, max_kf keyframes, max_kf * lm_stride landmark slots (256-B multiple). */
int64_t yv_map_block_bytes(int max_kf, int lm_stride);

/* yv_batch_track + the map block of this call's chunk: after the pose LM (on the same stream, so overlap mode
 * keeps the block off the critical path) the chunk's poses are composed (L_k) and every keyframe's LM inliers
 * (edge_outlier == 0) are written as landmarks. first_frame = global index of the batch's first track's frame;
 * d_block holds yv_map_block_bytes(max_kf, the batch's max_kp) bytes. */
int yv_batch_track_map(yv_batch* b, const double* d_priors, double* d_poses, int64_t first_frame, int kf_every,
                       void* d_block, int max_kf, void* stream);
/* `stream` waits for the block of the last yv_batch_track_map (e.g. the stream that runs the all-gather). */
int yv_batch_map_wait(yv_batch* b, void* stream);
/* The next yv_batch_track_map's block write waits for the work issued on `stream` so far (e.g. the all-gather
 * that reads the block): the caller releases the block once its readers are enqueued. Only the map kernels wait;
 * the edge build and the pose LM do not. */
int yv_batch_map_release(yv_batch* b, void* stream);

/* Place `world` gathered blocks (contiguous, block_bytes apart, in rank order) in world coordinates, in place, on
 * `stream`. d_base [7] (device, in / out): T_wc of the frame before block 0; on return T_wc of the last frame of
 * the last block. d_anchors [world][7] (device scratch, out: A_r). */
int yv_map_place(yv_ctx* ctx, void* d_blocks, int world, int64_t block_bytes, double* d_base, double* d_anchors,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* YAVO_MAP_H */

/*
 * yavo_oracle_map.c -- CPU restatement of the shared map blocks (include/yavo/yavo_map.h).
 *
 * TEST INFRASTRUCTURE ONLY (see yavo_oracle.h): the checker for ya_vo_amd/csrc/yavo_map.hip.
 *
 * The reference's map is one process-wide object: Map::insertKeyFrame keys frames by Frame::frameID and
 * Map::insertMapPoint keys landmarks by MapPoint::ptID (src/Map.cc:9-40, include/Map.hpp:12-13), with the
 * landmark position set from the triangulated point (src/LoopHandler.cc:676-697). A frame-sharded sequence builds
 * the same records per chunk: keyframe poses as the left fold of the chunk's relative poses (Sophus SE3d
 * products, or_se3_mul), landmarks as the pose LM's inliers in edge order, then places every chunk in world
 * coordinates by the serial anchor chain. "Parity unpinned" against the reference binary (it has no test for its
 * map and cannot be built here); the GPU kernels are checked against this file bit for bit.
 */
#include <stdint.h>
#include <string.h>

#include "../include/yavo/yavo_map.h"
#include "yavo_oracle.h"

static int64_t round256(int64_t x) { return (x + 255) & ~(int64_t)255; }
static int64_t lm_offset(int max_kf) {
    return round256((int64_t)sizeof(yv_map_header) + (int64_t)max_kf * (int64_t)sizeof(yv_keyframe));
}

int64_t or_map_block_bytes(int max_kf, int lm_stride) {
    if (max_kf < 1 || lm_stride < 1) return -1;
    return round256(lm_offset(max_kf) + (int64_t)max_kf * lm_stride * (int64_t)sizeof(yv_landmark));
}

/* One chunk's block. rel [n][7]: T_{k-1,k} per track (frame k-1's camera from frame k's); edge_count [n],
 * edge_X [n][max_kp][3] (frame k's left camera), edge_outlier [n][max_kp] (the LM's level flags). The block is
 * zeroed first so unwritten slots compare equal to a zero-initialised device block. */
void or_map_chunk(const double* rel, int n, int64_t first_frame, int kf_every, const int32_t* edge_count,
                  const double* edge_X, const uint8_t* edge_outlier, int max_kp, int max_kf, void* block) {
    uint8_t* b = (uint8_t*)block;
    memset(b, 0, (size_t)or_map_block_bytes(max_kf, max_kp));
    yv_map_header* h = (yv_map_header*)b;
    yv_keyframe* kf = (yv_keyframe*)(b + sizeof(yv_map_header));
    yv_landmark* lm = (yv_landmark*)(b + lm_offset(max_kf));
    double L[7] = {0, 0, 0, 1, 0, 0, 0};
    int n_kf = 0;
    for (int k = 0; k < n; ++k) {
        double T[7];
        if (k == 0)
            memcpy(T, rel, sizeof T); /* L_0 = rel_0 (no identity product) */
        else
            or_se3_mul(L, rel + 7 * k, T);
        memcpy(L, T, sizeof L);
        const int64_t g = first_frame + k;
        if (g % kf_every != 0 || n_kf >= max_kf) continue;
        yv_keyframe* f = kf + n_kf;
        f->frame_id = g;
        memcpy(f->T, L, sizeof L);
        yv_landmark* out = lm + (int64_t)n_kf * max_kp;
        int m = 0;
        for (int e = 0; e < edge_count[k]; ++e) {
            if (edge_outlier[(int64_t)k * max_kp + e] != 0) continue;
            out[m].id = (g << 16) | (int64_t)e; /* MapPoint::ptID: unique per (frame, edge) */
            memcpy(out[m].X, edge_X + ((int64_t)k * max_kp + e) * 3, 3 * sizeof(double));
            ++m;
        }
        f->n_landmarks = m;
        ++n_kf;
    }
    if (n > 0)
        memcpy(h->chunk, L, sizeof L);
    else {
        memset(h->chunk, 0, sizeof h->chunk);
        h->chunk[3] = 1.0;
    }
    h->first_frame = first_frame;
    h->n_frames = n;
    h->n_kf = n_kf;
    h->kf_every = kf_every;
    h->lm_stride = max_kp;
    h->max_kf = max_kf;
    h->placed = 0;
}

/* Placement of `world` gathered blocks: A_0 = base, A_{r+1} = A_r * C_r (blocks without frames keep the anchor);
 * keyframe T_wc = A_r * L_k, landmark X_w = T_wc * X. base <- A_world. */
void or_map_place(void* blocks, int world, int64_t bb, double* base, double* anchors) {
    uint8_t* all = (uint8_t*)blocks;
    double A[7];
    memcpy(A, base, sizeof A);
    for (int r = 0; r < world; ++r) {
        const yv_map_header* h = (const yv_map_header*)(all + r * bb);
        memcpy(anchors + 7 * r, A, sizeof A);
        if (h->n_frames > 0) {
            double T[7];
            or_se3_mul(A, h->chunk, T);
            memcpy(A, T, sizeof A);
        }
    }
    memcpy(base, A, sizeof A);
    for (int r = 0; r < world; ++r) {
        uint8_t* b = all + r * bb;
        yv_map_header* h = (yv_map_header*)b;
        yv_keyframe* kf = (yv_keyframe*)(b + sizeof(yv_map_header));
        yv_landmark* lm = (yv_landmark*)(b + lm_offset(h->max_kf));
        const int shard_world = h->placed >= 2;  /* a sequence shard's export: local T_wc, local-world X */
        for (int j = 0; j < h->n_kf; ++j) {
            double T[7];
            or_se3_mul(anchors + 7 * r, kf[j].T, T);
            memcpy(kf[j].T, T, sizeof T);
            yv_landmark* l = lm + (int64_t)j * h->lm_stride;
            for (int q = 0; q < kf[j].n_landmarks; ++q) {
                double Xw[3];
                or_se3_act(shard_world ? anchors + 7 * r : T, l[q].X, Xw);
                memcpy(l[q].X, Xw, sizeof Xw);
            }
        }
        if (h->n_kf > 0) h->placed = shard_world ? 3 : 1;
    }
}

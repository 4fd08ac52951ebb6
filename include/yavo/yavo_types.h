/*
 * yavo_types.h -- POD record layouts shared across the drop-in boundary.
 *
 * These are byte-identical to the reference's C++ classes so that a caller holding
 * std::vector<KeyPoint> / std::vector<Matches> can hand their .data() straight across:
 *
 *   class KeyPoint { int x; int y; int id; bool matched=false; uchar featVec[32]={}; };
 *       /root/reference/include/BriefDescriptor.hpp:11-24   -> 48 bytes (3 pad bytes at 45..47)
 *   class Matches  { KeyPoint pt1; KeyPoint pt2; int distance; };
 *       /root/reference/include/BriefDescriptor.hpp:27-39   -> 100 bytes
 *
 * Coordinate convention (parity-critical, kept from the reference): x = image ROW, y = image COLUMN
 * (FAST emits cv::Point(i, j) with i the row: src/FastDetector.cc:298-323).
 */
#ifndef YAVO_TYPES_H
#define YAVO_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct yv_keypoint {
    int32_t x;            /* row    (offset 0)  */
    int32_t y;            /* column (offset 4)  */
    int32_t id;           /* index into the detector output list (offset 8) */
    uint8_t matched;      /* bool  (offset 12) */
    uint8_t featVec[32];  /* 256-bit BRIEF descriptor, test j -> byte j>>3, bit j&7 (offset 13) */
    uint8_t _pad[3];      /* always written as zero by this library */
} yv_keypoint;

typedef struct yv_match {
    yv_keypoint pt1;      /* query keypoint (last frame), offset 0  */
    yv_keypoint pt2;      /* best train keypoint (x, y, id only), offset 48 */
    int32_t distance;     /* Hamming distance, INT_MAX when the train set is empty, offset 96 */
} yv_match;

#ifdef __cplusplus
}
#endif

#if defined(__cplusplus)
static_assert(sizeof(yv_keypoint) == 48, "yv_keypoint must match KeyPoint (48 B)");
static_assert(sizeof(yv_match) == 100, "yv_match must match Matches (100 B)");
#elif defined(__STDC_VERSION__) && __STDC_VERSION__ >= 201112L
_Static_assert(sizeof(yv_keypoint) == 48, "yv_keypoint must match KeyPoint (48 B)");
_Static_assert(sizeof(yv_match) == 100, "yv_match must match Matches (100 B)");
#endif

#endif /* YAVO_TYPES_H */

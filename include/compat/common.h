/* Compatibility header: lets sources written against fpgasystems/gcow sw/include (types.h, zfp.h, encode.h,
 * decode.h, stream.h, common.h) compile unchanged against libgcow.so. API constants and helper macros of
 * sw/include/common.h and types.h; every function comes from gcow.h. */
#ifndef GCOW_COMPAT_COMMON_H
#define GCOW_COMPAT_COMMON_H
#include <limits.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "gcow.h"

#define ZFP_MAGIC_BITS 32
#define ZFP_META_BITS 52
#define ZFP_MODE_SHORT_BITS 12
#define ZFP_MODE_LONG_BITS 64
#define ZFP_MODE_SHORT_MAX ((1u << ZFP_MODE_SHORT_BITS) - 2)
#define BLOCK_SIZE_2D 16
#define BLOCK_SIZE_4D 256
#define BLOCK_SIZE(dim) (1 << (2 * (dim)))
#ifndef MIN
#define MIN(x, y) ((x) < (y) ? (x) : (y))
#endif
#ifndef MAX
#define MAX(x, y) ((x) > (y) ? (x) : (y))
#endif
#define EBITS 8
#define EBIAS ((1 << (EBITS - 1)) - 1)
#define NBMASK 0xaaaaaaaau
#define SWORD_BITS ((size_t)(sizeof(stream_word) * CHAR_BIT))
#define FABS(x) (float)fabs(x)
#define FREXP(x, e) (void)frexp(x, e)
#define LDEXP(f, e) (float)ldexp(f, e)
#endif

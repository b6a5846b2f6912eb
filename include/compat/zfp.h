/* Compatibility header (see common.h): sw/include/zfp.h -> gcow.h */
#include "common.h"

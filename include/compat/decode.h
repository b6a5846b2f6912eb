/* Compatibility header (see common.h): sw/include/decode.h -> gcow.h */
#include "common.h"

/* Compatibility header (see common.h): sw/include/encode.h -> gcow.h */
#include "common.h"

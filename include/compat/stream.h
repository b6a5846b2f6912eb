/* Compatibility header (see common.h): sw/include/stream.h -> gcow.h */
#include "common.h"

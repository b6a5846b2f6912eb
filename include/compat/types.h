/* Compatibility header (see common.h): sw/include/types.h -> gcow.h */
#include "common.h"

// placeholder, filled in below
#include "common.h"

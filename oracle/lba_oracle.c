#include "lba_oracle.h"

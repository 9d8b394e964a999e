#include "orb_slam2_decls.h"  // test fixture: see orb_slam2_decls.h

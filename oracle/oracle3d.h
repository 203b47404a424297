// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h). 3D restatement.
#ifndef CSM_ORACLE3D_H_
#define CSM_ORACLE3D_H_
#include "csm_oracle.h"
#endif

#include <hip/hip_runtime.h>
#include <cstdio>
int main(){int lo=0,hi=0; hipDeviceGetStreamPriorityRange(&lo,&hi); printf("least %d greatest %d\n",lo,hi); return 0;}

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <time.h>
static double now(){struct timespec t; clock_gettime(CLOCK_MONOTONIC,&t); return t.tv_sec+t.tv_nsec*1e-9;}
int main(){ double t0=now(); int n=0; hipGetDeviceCount(&n); double t1=now(); void* p; hipMalloc(&p, 1<<20); double t2=now(); hipStream_t s; hipStreamCreate(&s); double t3=now();
 printf("{\"devcount_s\": %.4f, \"malloc_s\": %.4f, \"stream_s\": %.4f, \"n\": %d}\n", t1-t0, t2-t1, t3-t2, n); return 0; }

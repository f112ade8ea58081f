#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <time.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+t.tv_nsec*1e-9;}
int main(){
  size_t n=20u<<20; uint8_t *src=malloc(n), *dst=malloc(n), *pin;
  memset(src,1,n); memset(dst,0,n);
  hipHostMalloc((void**)&pin,n,hipHostMallocDefault); memset(pin,0,n);
  for(int r=0;r<3;r++){
    double t0=now(); memcpy(dst,src,n); double t1=now(); memcpy(pin,src,n); double t2=now(); memcpy(dst,pin,n); double t3=now();
    uint64_t *o=(uint64_t*)src, *po=(uint64_t*)pin; double t4=now(); for(size_t i=0;i<n/8;i++) po[i]=o[i]-1; double t5=now();
    printf("{\"heap_to_heap_ms\": %.3f, \"heap_to_pinned_ms\": %.3f, \"pinned_to_heap_ms\": %.3f, \"rebase_into_pinned_ms\": %.3f}\n",(t1-t0)*1e3,(t2-t1)*1e3,(t3-t2)*1e3,(t5-t4)*1e3);
  }
  return 0;
}

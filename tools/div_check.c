// Markstein-corrected division vs IEEE x / d (common.hpp div_rn): gcc -O2 -ffp-contract=off tools/div_check.c -lm
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float f(uint32_t u){float x; memcpy(&x,&u,4); return x;}
int main(){
  uint64_t bad=0, tot=0; uint32_t s=12345;
  for(int d=1; d<=1024; ++d){
    volatile float df=(float)d; float r = 1.0f/df;
    for(int i=0;i<2000000;++i){
      s = s*1664525u+1013904223u; uint32_t e = 1 + (s>>8)%252; // normal exponents (no subnormal/inf)
      uint32_t s2 = s*22695477u+1u;
      uint32_t u = ((s2&1)<<31) | (e<<23) | ((s2>>9)&0x7fffff);
      float x = f(u);
      volatile float q0 = x*r; float rem = fmaf(-q0, df, x); float q = fmaf(rem, r, q0);
      float ref = x/df;
      tot++; if (fabsf(ref) >= 0x1p-126f && q != ref && !(isinf(ref)&&isinf(q))) { if(bad<5) printf("x=%a d=%d q=%a ref=%a\n",x,d,q,ref); bad++; }
    }
  }
  printf("bad %llu of %llu\n",(unsigned long long)bad,(unsigned long long)tot);
}

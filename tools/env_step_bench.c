/* Times the native env stepper (csrc/envstep.c) alone: 64 envs, hopper dims.
 *   gcc -O3 -march=x86-64-v3 -o tools/env_step_bench tools/env_step_bench.c diffusionpolicyoptimization_amd/csrc/envstep.c */
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>
int dppo_env_step(int E, int Do, int Da, int act_steps, int Ta, int max_steps, int n_obs_steps,
 const double* AT, const double* B, const double* c, const double* goal, double* state, int64_t* cnt, const float* actions,
 double* reward, uint8_t* terminated, uint8_t* truncated, float* obs_out);
int main(){int E=64,Do=11,Da=3; double *AT=calloc(Do*Do,8),*B=calloc(Da*Do,8),*c=calloc(Do,8),*g=calloc(Do,8),*st=calloc(E*Do,8),*rw=calloc(E,8);
int64_t*cnt=calloc(E,8); float*a=calloc(E*4*Da,4),*o=calloc(E*Do,4); uint8_t*t1=calloc(E,1),*t2=calloc(E,1);
for(int i=0;i<Do*Do;i++)AT[i]=0.01*i;
struct timespec s,e; for(int r=0;r<1000;r++) dppo_env_step(E,Do,Da,4,4,1000000000,1,AT,B,c,g,st,cnt,a,rw,t1,t2,o);
clock_gettime(CLOCK_MONOTONIC,&s); int n=100000; for(int r=0;r<n;r++) dppo_env_step(E,Do,Da,4,4,1000000000,1,AT,B,c,g,st,cnt,a,rw,t1,t2,o);
clock_gettime(CLOCK_MONOTONIC,&e); printf("C env step: %.2f us\n", ((e.tv_sec-s.tv_sec)*1e9+(e.tv_nsec-s.tv_nsec))/n/1e3);}

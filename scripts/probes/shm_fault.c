// Cost of first-touch page faults on a /dev/shm mapping (object-store writes/reads).
#define _GNU_SOURCE
#include <sys/mman.h>
#include <fcntl.h>
#include <unistd.h>
#include <string.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec*1e3+t.tv_nsec/1e6;}
int main(){
  size_t S=1ul<<30, N=36ul<<20;
  int fd=open("/dev/shm/ra_shm_fault_probe",O_RDWR|O_CREAT|O_TRUNC,0600); if(ftruncate(fd,S))return 1;
  char* src=malloc(N); memset(src,1,N);
  char* p=mmap(0,S,PROT_READ|PROT_WRITE,MAP_SHARED,fd,0);
  double t0,t1,t2; volatile long s=0; int rc;
  t0=now(); memcpy(p,src,N); t1=now(); memcpy(p,src,N); t2=now();
  printf("A fresh memcpy %.2f ms, same pages again %.2f ms\n",t1-t0,t2-t1);
  t0=now(); rc=madvise(p+N,N,MADV_POPULATE_WRITE); t1=now(); memcpy(p+N,src,N); t2=now();
  printf("B fresh: populate_write(rc=%d) %.2f + memcpy %.2f\n",rc,t1-t0,t2-t1);
  if(fallocate(fd,0,2*N,3*N)) perror("fallocate");
  t0=now(); memcpy(p+2*N,src,N); t1=now();
  printf("C fallocated, memcpy %.2f\n",t1-t0);
  char* q=mmap(0,S,PROT_READ|PROT_WRITE,MAP_SHARED,fd,0);  // "another process": allocated, unmapped
  t0=now(); memcpy(q,src,N); t1=now(); printf("D other mapping memcpy %.2f\n",t1-t0);
  t0=now(); for(size_t i=0;i<N;i+=4096)s+=q[N+i]; t1=now(); memcpy(q+N,src,N); t2=now();
  printf("E other mapping read-touch %.2f + memcpy %.2f\n",t1-t0,t2-t1);
  t0=now(); rc=madvise(q+2*N,N,MADV_POPULATE_READ); t1=now(); memcpy(q+2*N,src,N); t2=now();
  printf("F other mapping populate_read(rc=%d) %.2f + memcpy %.2f\n",rc,t1-t0,t2-t1);
  t0=now(); rc=madvise(q+3*N,N,MADV_POPULATE_WRITE); t1=now(); memcpy(q+3*N,src,N); t2=now();
  printf("G other mapping populate_write(rc=%d) %.2f + memcpy %.2f\n",rc,t1-t0,t2-t1);
  t0=now(); rc=fallocate(fd,0,8*N,8*N); t1=now(); printf("H fallocate 8x36MB %.2f ms rc=%d\n",t1-t0,rc);
  char* r=mmap(0,S,PROT_READ|PROT_WRITE,MAP_SHARED,fd,0);
  t0=now(); rc=madvise(r+20*N,N,MADV_POPULATE_READ); t1=now(); memcpy(r+20*N,src,N); t2=now();
  printf("I fresh hole: populate_read(rc=%d) %.2f + memcpy %.2f\n",rc,t1-t0,t2-t1);
  t0=now(); rc=madvise(r+9*N,N,MADV_POPULATE_READ); t1=now(); memcpy(r+9*N,src,N); t2=now();
  printf("J fallocated: populate_read(rc=%d) %.2f + memcpy %.2f\n",rc,t1-t0,t2-t1);
  unlink("/dev/shm/ra_shm_fault_probe"); return 0;}

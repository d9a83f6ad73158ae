#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
static uint32_t fb(float f){uint32_t u;memcpy(&u,&f,4);return u;}
int main(){
  srand(1);
  int n=2560,K=8,L=n/K; int hist[200]={0}; int maxd=0; long tot=0, miss16=0, miss32=0;
  for(int trial=0;trial<20000;trial++){
    float x[2560];
    double scale = exp((rand()/(double)RAND_MAX-0.5)*10);
    for(int i=0;i<n;i++){ double u1=(rand()+1.0)/(RAND_MAX+2.0),u2=rand()/(double)RAND_MAX; x[i]=(float)(scale*sqrt(-2*log(u1))*cos(2*M_PI*u2)); if (trial%3==0) x[i]*= (i%97==0)?50:1; }
    float s=0; double p=0;
    for(int k=0;k<K;k++){
      if(k>0){ float est=(float)p; int d=(int)fb(s)-(int)fb(est); if(abs(d)>maxd)maxd=abs(d); tot++; if(d< -16||d>=16)miss16++; if(d<-32||d>=32)miss32++; int b=d+100; if(b<0)b=0; if(b>199)b=199; hist[b]++; }
      for(int i=k*L;i<(k+1)*L;i++){ s=fmaf(x[i],x[i],s); p+=(double)x[i]*x[i]; }
    }
  }
  printf("boundaries %ld maxd %d miss16 %ld miss32 %ld\n",tot,maxd,miss16,miss32);
  for(int b=80;b<120;b++) printf("%d:%d ",b-100,hist[b]); printf("\n");
}

// biquad_state_sync.c -- how soon two DF-I biquad trajectories (fp32, no FMA
// contraction, biquad.cpp's arithmetic) from different States agree bit for bit on
// the same input: the warm-up the speculative segments of a State-writing plugin
// need.  gcc -O2 -ffp-contract=off biquad_state_sync.c -lm
// usage: ./a.out cutoff_hz q [input_scale]
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
// two DF-I biquad trajectories (fp32, no contraction) from different states; when do they agree bitwise?
static uint64_t st=88172645463325252ull; static float rnd(){ st^=st<<13; st^=st>>7; st^=st<<17; return (float)((st>>40)/(double)(1<<24))*2.f-1.f; }
int main(int argc,char**argv){
  double fc=atof(argv[1]), q=atof(argv[2]); int trials=200; double sr=48000;
  double w0=2*M_PI*fc/sr, al=sin(w0)/(2*q), c=cos(w0), a0=1+al;
  float b0=(float)((1-c)/2/a0), b1=(float)((1-c)/a0), b2=b0, a1=(float)(-2*c/a0), a2=(float)((1-al)/a0);
  long worst=0, sum=0, fail=0;
  for(int t=0;t<trials;t++){
    float x1=0,x2=0,y1=0,y2=0, X1=rnd(),X2=rnd(),Y1=rnd()*3,Y2=rnd()*3; // warm-up guess vs truth
    long n; long N=1<<22;
    for(n=0;n<N;n++){ float x=rnd()*(argc>3?atof(argv[3]):1.f);
      volatile float p0=b0*x, p1=b1*x1, p2=b2*x2, p3=a1*y1, p4=a2*y2; float y=p0+p1+p2-p3-p4;
      volatile float P1=b1*X1, P2=b2*X2, P3=a1*Y1, P4=a2*Y2; float Y=p0+P1+P2-P3-P4;
      x2=x1;x1=x;y2=y1;y1=y; X2=X1;X1=x;Y2=Y1;Y1=Y;
      if(y1==Y1&&y2==Y2&&x1==X1&&x2==X2) break; }
    if(n==N) fail++; else { sum+=n; if(n>worst) worst=n; }
  }
  printf("fc %g q %g: synced %d/%d, mean %ld, worst %ld samples\n",fc,q,trials-(int)fail,trials,trials>fail?sum/(trials-fail):0,worst);
}

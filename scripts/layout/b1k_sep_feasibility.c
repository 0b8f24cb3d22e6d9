// br1024 spectrum layout: exhaustive check that no sum-separable octal-digit slot table S0[d0] + S1[d1] + S2[d2]
// makes both the pass-0 / MAC b128 reads (4 x 16-lane groups, slot mod 16) and the pass-2 b128 writes
// (8-lane groups, slot mod 8) conflict-free: the read partitions of Z16 force B0..B3 (= S1 mod 16) into
// at most two classes mod 8, the writes need eight.  gcc -O2 b1k_sep_feasibility.c && ./a.out -> found 0
#include <stdio.h>
int main(){
  long found=0;
  for(int xm=0;xm<256;xm++){ // choose which 4 residues mod 8 go to X
    if(__builtin_popcount(xm)!=4) continue;
    int xr[4],yr[4],nx=0,ny=0;
    for(int r=0;r<8;r++){ if(xm>>r&1) xr[nx++]=r; else yr[ny++]=r; }
    for(int xh=0;xh<16;xh++) for(int yh=0;yh<16;yh++){
      unsigned X=0,Y=0;
      for(int i=0;i<4;i++){ X|=1u<<(xr[i]+8*((xh>>i)&1)); Y|=1u<<(yr[i]+8*((yh>>i)&1)); }
      // rotations
      unsigned Xs[16],Ys[16];
      for(int b=0;b<16;b++){ Xs[b]=((X<<b)|(X>>(16-b)))&0xFFFF; Ys[b]=((Y<<b)|(Y>>(16-b)))&0xFFFF; }
      for(int b0=0;b0<16;b0++) for(int b3=0;b3<16;b3++){
        if((b0&7)==(b3&7)) continue;
        if(Xs[b0]&Xs[b3]) continue; if(Ys[b0]&Ys[b3]) continue;
        for(int b1=0;b1<16;b1++){ if((b1&7)==(b0&7)||(b1&7)==(b3&7)) continue;
          if((Xs[b0]|Xs[b3])&Ys[b1]) continue; if((Ys[b0]|Ys[b3])&Xs[b1]) continue;
          for(int b2=0;b2<16;b2++){ if((b2&7)==(b0&7)||(b2&7)==(b3&7)||(b2&7)==(b1&7)) continue;
            if(((Xs[b0]|Xs[b3]|Ys[b1]|Ys[b2])==0xFFFF) && ((Ys[b0]|Ys[b3]|Xs[b1]|Xs[b2])==0xFFFF)){
              if(found<5) printf("X=%04x Y=%04x B=%d %d %d %d\n",X,Y,b0,b1,b2,b3);
              found++;
            }
          }
        }
      }
    }
  }
  printf("found %ld\n",found);
}

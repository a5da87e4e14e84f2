// scripts/leafbvh_harness.cpp — host-side cost model of the leaf BVH walk.
// Builds csrc/pt_leafbvh.cpp's tree over one leaf's records (a file of 48-byte Tri records, e.g.
// the boat's 7327-entry leaf) and replays the walk's skip rule in float for 2000 random rays:
// entry tests and nodes per ray (per-lane walk), why nodes stay open, the cone histogram, and a
// cooperative variant (one ray, 64 lanes over a level-synchronous frontier) in wave-steps.
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off
//        -I brown-cs2240-path-tracer_amd/csrc scripts/leafbvh_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
#include <hip/hip_runtime.h>
#include "pt_leafbvh.h"
#include <cstdio>
#include <cmath>
#include <random>
#include <vector>
using namespace pt;
// walk simulation in float, same rule as pt_device.h leaf_walk (no tie detail needed for stats)
static bool tri_hit(const Tri& T, const float o[3], const float d[3], float& t) {
    float e1[3]={T.q0[3],T.q1[0],T.q1[1]}, e2[3]={T.q1[2],T.q1[3],T.e2z}, v0[3]={T.q0[0],T.q0[1],T.q0[2]};
    float h[3]={d[1]*e2[2]-d[2]*e2[1], d[2]*e2[0]-d[0]*e2[2], d[0]*e2[1]-d[1]*e2[0]};
    float det=e1[0]*h[0]+e1[1]*h[1]+e1[2]*h[2];
    if (det>-1e-8f && det<1e-8f) return false;
    float inv=1.0f/det; float s[3]={o[0]-v0[0],o[1]-v0[1],o[2]-v0[2]};
    float u=inv*(s[0]*h[0]+s[1]*h[1]+s[2]*h[2]); if(u<0||u>1) return false;
    float q[3]={s[1]*e1[2]-s[2]*e1[1], s[2]*e1[0]-s[0]*e1[2], s[0]*e1[1]-s[1]*e1[0]};
    float v=inv*(d[0]*q[0]+d[1]*q[1]+d[2]*q[2]); if(v<0||u+v>1) return false;
    t=inv*(e2[0]*q[0]+e2[1]*q[1]+e2[2]*q[2]); return t>1e-8f;
}
int main(int argc, char** argv) {
    FILE* f=fopen(argv[1],"rb"); std::vector<Tri> tris; Tri t;
    while (fread(&t,sizeof t,1,f)==1) tris.push_back(t); fclose(f);
    int n=(int)tris.size();
    std::vector<LNode> nodes; std::vector<int32_t> lidx; int32_t root,end;
    build_leaf_bvh(tris.data(),0,n,nodes,lidx,root,end);
    printf("entries %d nodes %d\n", n, end-root);
    std::mt19937 rng(5); std::uniform_real_distribution<float> U(0,1); std::normal_distribution<float> N(0,1);
    double coop=0,tests=0,nv=0,bad=0,ncone=0,ndl=0,nbox=0; double sa_hist[10]={0}; int R=2000;
    for (int r=0;r<R;++r) {
        int k=rng()%n; float bu=U(rng),bv=U(rng); if(bu+bv>1){bu=1-bu;bv=1-bv;}
        const Tri& T=tris[k]; float P[3]={T.q0[0]+bu*T.q0[3]+bv*T.q1[2], T.q0[1]+bu*T.q1[0]+bv*T.q1[3], T.q0[2]+bu*T.q1[1]+bv*T.e2z};
        float o[3]={P[0]+10*U(rng)-5,P[1]+10*U(rng)-5,P[2]+10*U(rng)-5}, d[3]={N(rng),N(rng),N(rng)};
        float l=std::sqrt(d[0]*d[0]+d[1]*d[1]+d[2]*d[2]); for(int a=0;a<3;++a) d[a]/=l;
        float inv[3]={1.0f/d[0],1.0f/d[1],1.0f/d[2]};
        float on=std::sqrt(o[0]*o[0]+o[1]*o[1]+o[2]*o[2]);
        float bt=INFINITY; int bk=0x7fffffff; int i=root;
        float lt=INFINITY; for(int j=0;j<n;++j){float tt; if(tri_hit(tris[j],o,d,tt)&&tt<lt) lt=tt;}
        while(i<end){
            const LNode& q=nodes[i]; nv++;
            float cb=std::fabs(d[0]*q.ax+d[1]*q.ay+d[2]*q.az); float sb=std::sqrt(std::fmax(0.f,1-cb*cb));
            float cf=cb*q.ca-sb*q.sa-1e-5f; bool skip=false;
            if(!(cf>1e-4f)) { ncone++; int b=(int)(q.sa*9.99f); sa_hist[b]++; }
            if(cf>1e-4f){ float dl=(q.A+q.B*on)/cf+1e-5f*on+q.C; if(dl<1e30f){ float tn=-3e38f,tf=3e38f;
                for(int a=0;a<3;++a){float t1=(q.lo[a]-dl-o[a])*inv[a],t2=(q.hi[a]+dl-o[a])*inv[a]; tn=std::fmax(tn,std::fmin(t1,t2)); tf=std::fmin(tf,std::fmax(t1,t2));}
                skip=(tf<tn)||(tf<0)||(tn>bt); if(!skip) nbox++;} else ndl++;}
            if(!skip && q.info>=0){int first=q.info&0xffffff,c=q.info>>24; for(int j=0;j<c;++j){int kk=lidx[first+j]; float tt; tests++; if(tri_hit(tris[kk],o,d,tt)&&(tt<bt||(tt==bt&&kk<bk))){bt=tt;bk=kk;}}}
            i=(!skip&&q.info<0)?i+1:q.skip;
        }
        if (!(bt==lt || (std::isinf(bt)&&std::isinf(lt)))) bad++;
        { // cooperative: one ray, 64 lanes over a frontier (level-synchronous); wave-steps
          std::vector<int> fr, nx; for (int j=root;j<end;){ fr.push_back(j); j=nodes[j].skip; }
          float cb2=INFINITY; double steps=0;
          while(!fr.empty()){
            nx.clear();
            for (size_t c=0;c<fr.size();c+=64){
              int maxtests=0;
              for (size_t z=c; z<std::min(fr.size(),c+64); ++z){
                const LNode& q=nodes[fr[z]];
                float cb=std::fabs(d[0]*q.ax+d[1]*q.ay+d[2]*q.az); float sb=std::sqrt(std::fmax(0.f,1-cb*cb));
                float cf=cb*q.ca-sb*q.sa-1e-5f; bool skip=false;
                if(cf>1e-4f){ float dl=(q.A+q.B*on)/cf+1e-5f*on+q.C; if(dl<1e30f){ float tn=-3e38f,tf=3e38f;
                    for(int a=0;a<3;++a){float t1=(q.lo[a]-dl-o[a])*inv[a],t2=(q.hi[a]+dl-o[a])*inv[a]; tn=std::fmax(tn,std::fmin(t1,t2)); tf=std::fmin(tf,std::fmax(t1,t2));}
                    skip=(tf<tn)||(tf<0)||(tn>cb2);}}
                if(skip) continue;
                if(q.info>=0){int first=q.info&0xffffff,cn=q.info>>24; maxtests=std::max(maxtests,cn); for(int j=0;j<cn;++j){float tt; if(tri_hit(tris[lidx[first+j]],o,d,tt)&&tt<cb2) cb2=tt;}}
                else { nx.push_back(fr[z]+1); nx.push_back(nodes[fr[z]+1].skip); }
              }
              steps += 1 + maxtests;
            }
            std::swap(fr,nx);
          }
          coop += steps;
        }
    }
    printf("per ray: tests %.1f nodes %.1f mismatches %.0f  open: cone %.1f dl %.1f box %.1f\n", tests/R, nv/R, bad, ncone/R, ndl/R, nbox/R);
    printf("cooperative wave-steps per ray %.1f (brute %d)\n", coop/R, (n+63)/64);
    for(int b=0;b<10;++b) printf("sa %.1f: %.1f\n", b/10.0, sa_hist[b]/R);
    // node cone distribution
    int hist[10]={0}; for (auto& q: nodes) hist[(int)(q.sa*9.99f)]++;
    for(int b=0;b<10;++b) printf("nodes with sa in [%.1f,%.1f): %d\n", b/10.0,(b+1)/10.0,hist[b]);
}

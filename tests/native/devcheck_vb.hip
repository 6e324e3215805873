// TEST-ONLY device harness for the batched-verification kernels: includes vbatch.hip as compiled
// in the product and drives its launchers, so a test can read the intermediate arrays
// (decompressed points, combined points) back.  Never loaded by the product.
#include "../../charon_amd/csrc/vbatch.hip"

using namespace hb;

// decompress, item->group, k_rlc; returns the combined points as raw Jacobian limbs
extern "C" int dc_vb_rlc(const uint8_t* pks, const uint8_t* sigs, uint32_t n, const uint32_t* grp_off,
                         uint32_t n_groups, const uint32_t* key8, uint8_t* pr_raw, uint8_t* sr_raw, uint8_t* gp_raw,
                         uint8_t* gst_out) {
  uint8_t *dpk, *dsig, *pst, *sst;
  G1AEntry* vpk;
  HmEntry* vsig;
  uint32_t *dgo, *ig;
  G1JEntry* pr;
  G2JEntry* sr;
  if (hipMalloc(&dpk, 48 * n) || hipMalloc(&dsig, 96 * n) || hipMalloc(&pst, n) || hipMalloc(&sst, n) ||
      hipMalloc(&vpk, sizeof(G1AEntry) * n) || hipMalloc(&vsig, sizeof(HmEntry) * n) ||
      hipMalloc(&dgo, 4 * (n_groups + 1)) || hipMalloc(&ig, 4 * n) || hipMalloc(&pr, sizeof(G1JEntry) * n) ||
      hipMalloc(&sr, sizeof(G2JEntry) * n))
    return -1;
  hipMemset(pr, 0, sizeof(G1JEntry) * n);
  hipMemset(sr, 0, sizeof(G2JEntry) * n);
  hipMemcpy(dpk, pks, 48 * n, hipMemcpyHostToDevice);
  hipMemcpy(dsig, sigs, 96 * n, hipMemcpyHostToDevice);
  hipMemcpy(dgo, grp_off, 4 * (n_groups + 1), hipMemcpyHostToDevice);
  RlcKey key;
  for (int k = 0; k < 8; k++) key.w[k] = key8[k];
  launch_dec_pk(dpk, n, vpk, pst, 0);
  launch_dec_sig_pt(dsig, n, vsig, sst, 0);
  launch_item_group(dgo, n_groups, n, ig, 0);
  launch_rlc(vpk, pst, vsig, sst, ig, dgo, 0, n, 0, key, pr, sr, 0);
  // group prep (message table: one zero entry, not used by the sums)
  MsgEntry* hm;
  G1AEntry* gP;
  uint8_t* gst;
  uint32_t *gmsg, *midx;
  LineEntry* gl;
  if (hipMalloc(&hm, sizeof(MsgEntry)) || hipMalloc(&gP, sizeof(G1AEntry) * n_groups) || hipMalloc(&gst, n_groups) ||
      hipMalloc(&gmsg, 4 * n_groups) || hipMalloc(&midx, 4 * n) || hipMalloc(&gl, sizeof(LineEntry) * N_LINES * n_groups))
    return -1;
  hipMemset(hm, 0, sizeof(MsgEntry));
  hipMemset(midx, 0, 4 * n);
  GroupPrepArgs ga{};
  ga.grp_off = dgo;
  ga.g0 = 0;
  ga.ng = n_groups;
  ga.msg_idx = midx;
  ga.hm = hm;
  ga.pk = vpk;
  ga.pk_st = pst;
  ga.sig = vsig;
  ga.sig_st = sst;
  ga.pr = pr;
  ga.sr = sr;
  ga.gP = gP;
  ga.gmsg = gmsg;
  ga.gst = gst;
  ga.glines = gl;
  launch_group_prep(ga, 0);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  hipMemcpy(gp_raw, gP, sizeof(G1AEntry) * n_groups, hipMemcpyDeviceToHost);
  hipMemcpy(gst_out, gst, n_groups, hipMemcpyDeviceToHost);
  hipMemcpy(pr_raw, pr, sizeof(G1JEntry) * n, hipMemcpyDeviceToHost);
  hipMemcpy(sr_raw, sr, sizeof(G2JEntry) * n, hipMemcpyDeviceToHost);
  for (void* p : {(void*)dpk, (void*)dsig, (void*)pst, (void*)sst, (void*)vpk, (void*)vsig, (void*)dgo, (void*)ig,
                  (void*)pr, (void*)sr})
    hipFree(p);
  return 0;
}

// one lane sums the raw Jacobian G1 points pr[0..n) (a loop like k_group_prep's) and, separately,
// the first two (straight-line), then compresses both
__global__ void k_dc_sum(const G1JEntry* pr, uint32_t n, uint8_t* out48, uint8_t* out48b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (threadIdx.x != 0) return;
  G1J acc = jac_infinity<Fp>();
  for (uint32_t i = 0; i < n; i++) {
    const G1JEntry pj = pr[i];
    acc = jac_add(acc, G1J{pj.X, pj.Y, pj.Z});
  }
  uint8_t b[48];
  g1_compress(b, jac_to_aff(acc));
  for (int k = 0; k < 48; k++) out48[k] = b[k];
  const G1JEntry p0 = pr[0], p1 = pr[1];
  g1_compress(b, jac_to_aff(jac_add(G1J{p0.X, p0.Y, p0.Z}, G1J{p1.X, p1.Y, p1.Z})));
  for (int k = 0; k < 48; k++) out48b[k] = b[k];
#endif
}

extern "C" int dc_sum(const uint8_t* pr_raw, uint32_t n, uint8_t* out48, uint8_t* out48b) {
  G1JEntry* pr;
  uint8_t *o, *ob;
  if (hipMalloc(&pr, sizeof(G1JEntry) * n) || hipMalloc(&o, 48) || hipMalloc(&ob, 48)) return -1;
  hipMemcpy(pr, pr_raw, sizeof(G1JEntry) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_dc_sum, dim3(1), dim3(64), 0, 0, pr, n, o, ob);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  hipMemcpy(out48, o, 48, hipMemcpyDeviceToHost);
  hipMemcpy(out48b, ob, 48, hipMemcpyDeviceToHost);
  hipFree(pr);
  hipFree(o);
  hipFree(ob);
  return 0;
}

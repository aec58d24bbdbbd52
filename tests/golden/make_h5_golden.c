/* Writes the Keras weight-file fixtures of tests/golden/ with the real HDF5 library (libhdf5, default
 * file-creation properties, as h5py uses them), so that the pure-Python HDF5 reader/writer of
 * adipose_amd/h5io.py is pinned to an independent implementation of the format.
 *
 *   keras_v3.weights.h5       Keras 2.13 saving_lib weights-only layout (model.save_weights to
 *                             *.weights.h5): /vars (model's own, empty), /layers/<name>/vars/<i>,
 *                             plus /optimizer/vars/0 (an int64 iteration counter) and an empty
 *                             /layers/input_layer/vars (layers without weights)
 *   keras_legacy.h5           legacy hdf5_format (model.save_weights to *.h5): root attrs layer_names,
 *                             backend, keras_version; <layer> attr weight_names; datasets
 *                             <layer>/<layer>/kernel:0 and bias:0
 *   keras_legacy_model.h5     the same under a /model_weights group (model.save to *.h5)
 *
 * Values: kernel element i = 0.001*i - 0.25, bias element i = 0.5*i + 0.125 (float32), so that tests
 * recompute them. Build + run (this container; the HDF5 C library ships in /opt/conda):
 *   gcc tests/golden/make_h5_golden.c -I/opt/conda/include -L/opt/conda/lib -lhdf5 \
 *       -Wl,-rpath,/opt/conda/lib -o /tmp/make_h5_golden && /tmp/make_h5_golden tests/golden
 */
#include <stdio.h>
#include <string.h>
#include "hdf5.h"

typedef struct { const char* name; int rank; hsize_t kdims[4]; int bias; } Layer;
static const Layer LAYERS[] = {
    {"down1_conv1", 4, {3, 3, 1, 4}, 4},
    {"dilate2", 4, {3, 3, 4, 4}, 4},
    {"main_out", 4, {1, 1, 4, 2}, 2},
};
static const int NL = 3;

static void fill(float* v, hsize_t n, int bias) {
  for (hsize_t i = 0; i < n; ++i) v[i] = bias ? 0.5f * (float)i + 0.125f : 0.001f * (float)i - 0.25f;
}

static void dataset(hid_t loc, const char* name, int rank, const hsize_t* dims, int bias) {
  hsize_t n = 1;
  for (int i = 0; i < rank; ++i) n *= dims[i];
  float buf[4096];
  fill(buf, n, bias);
  hid_t sp = H5Screate_simple(rank, dims, NULL);
  hid_t lcpl = H5Pcreate(H5P_LINK_CREATE);
  H5Pset_create_intermediate_group(lcpl, 1);
  hid_t d = H5Dcreate2(loc, name, H5T_IEEE_F32LE, sp, lcpl, H5P_DEFAULT, H5P_DEFAULT);
  H5Dwrite(d, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf);
  H5Dclose(d);
  H5Pclose(lcpl);
  H5Sclose(sp);
}

/* fixed-length NULLPAD string array attribute (what h5py writes for a numpy 'S' array) */
static void str_attr(hid_t loc, const char* name, const char** vals, int n) {
  size_t len = 1;
  for (int i = 0; i < n; ++i) if (strlen(vals[i]) > len) len = strlen(vals[i]);
  char buf[64 * 64];
  memset(buf, 0, sizeof(buf));
  for (int i = 0; i < n; ++i) memcpy(buf + i * len, vals[i], strlen(vals[i]));
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, len);
  H5Tset_strpad(t, H5T_STR_NULLPAD);
  hsize_t dims[1] = {(hsize_t)n};
  hid_t sp = H5Screate_simple(1, dims, NULL);
  hid_t a = H5Acreate2(loc, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
  H5Awrite(a, t, buf);
  H5Aclose(a);
  H5Sclose(sp);
  H5Tclose(t);
}

static void scalar_str_attr(hid_t loc, const char* name, const char* val) {
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, strlen(val));
  H5Tset_strpad(t, H5T_STR_NULLPAD);
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t a = H5Acreate2(loc, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
  H5Awrite(a, t, val);
  H5Aclose(a);
  H5Sclose(sp);
  H5Tclose(t);
}

static void legacy(hid_t root) {
  const char* names[3];
  for (int l = 0; l < NL; ++l) names[l] = LAYERS[l].name;
  str_attr(root, "layer_names", names, NL);
  scalar_str_attr(root, "backend", "tensorflow");
  scalar_str_attr(root, "keras_version", "2.13.1");
  for (int l = 0; l < NL; ++l) {
    hid_t g = H5Gcreate2(root, LAYERS[l].name, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    char k[128], b[128];
    snprintf(k, sizeof k, "%s/kernel:0", LAYERS[l].name);
    snprintf(b, sizeof b, "%s/bias:0", LAYERS[l].name);
    const char* wn[2] = {k, b};
    str_attr(g, "weight_names", wn, 2);
    dataset(g, k, LAYERS[l].rank, LAYERS[l].kdims, 0);
    hsize_t bd[1] = {(hsize_t)LAYERS[l].bias};
    dataset(g, b, 1, bd, 1);
    H5Gclose(g);
  }
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  char path[512];

  snprintf(path, sizeof path, "%s/keras_v3.weights.h5", dir);
  hid_t f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  H5Gclose(H5Gcreate2(f, "vars", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
  hid_t lcpl = H5Pcreate(H5P_LINK_CREATE);
  H5Pset_create_intermediate_group(lcpl, 1);
  H5Gclose(H5Gcreate2(f, "layers/input_layer/vars", lcpl, H5P_DEFAULT, H5P_DEFAULT));
  for (int l = 0; l < NL; ++l) {
    char p[256];
    snprintf(p, sizeof p, "layers/%s/vars/0", LAYERS[l].name);
    dataset(f, p, LAYERS[l].rank, LAYERS[l].kdims, 0);
    snprintf(p, sizeof p, "layers/%s/vars/1", LAYERS[l].name);
    hsize_t bd[1] = {(hsize_t)LAYERS[l].bias};
    dataset(f, p, 1, bd, 1);
  }
  {
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t d = H5Dcreate2(f, "optimizer/vars/0", H5T_STD_I64LE, sp, lcpl, H5P_DEFAULT, H5P_DEFAULT);
    long long it = 1234;
    H5Dwrite(d, H5T_NATIVE_LLONG, H5S_ALL, H5S_ALL, H5P_DEFAULT, &it);
    H5Dclose(d);
    H5Sclose(sp);
  }
  H5Pclose(lcpl);
  H5Fclose(f);

  snprintf(path, sizeof path, "%s/keras_legacy.h5", dir);
  f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  legacy(f);
  H5Fclose(f);

  snprintf(path, sizeof path, "%s/keras_legacy_model.h5", dir);
  f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  hid_t mw = H5Gcreate2(f, "model_weights", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  legacy(mw);
  H5Gclose(mw);
  H5Fclose(f);
  printf("wrote fixtures to %s\n", dir);
  return 0;
}

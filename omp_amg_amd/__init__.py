"""omp_amg_amd: MI355X-native AMG setup (HIP) behind the gslib crs/amg_setup C ABI."""

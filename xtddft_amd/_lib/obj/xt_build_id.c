static const char id[] = "XT_BUILD_ID:8d13ecbb9d581cf5e109f86b35e71079";
const char* xt_build_id(void) { return id + 12; }

static const char id[] = "XT_BUILD_ID:5079571588f33adcf6424e9918988edf";
const char* xt_build_id(void) { return id + 12; }

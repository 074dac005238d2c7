extern "C" const char* gpi_source_sha(void) { return "e8b146c63c2287877936c73f42701879bfac0c1f"; }

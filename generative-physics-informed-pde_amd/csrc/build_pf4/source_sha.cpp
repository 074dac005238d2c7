extern "C" const char* gpi_source_sha(void) { return "e16683154faa17501e0c7e499b6295d5a14cae75"; }

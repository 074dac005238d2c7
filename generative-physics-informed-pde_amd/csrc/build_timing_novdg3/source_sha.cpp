extern "C" const char* gpi_source_sha(void) { return "ca46497efb98ec6a2b9f901bc1541a88c22cd3fa"; }

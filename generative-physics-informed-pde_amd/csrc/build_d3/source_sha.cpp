extern "C" const char* gpi_source_sha(void) { return "affa6b66e18b4558afbc4bb738844e97589162bd"; }

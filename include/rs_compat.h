/*
 * rs_compat.h -- link-compatible drop-in for UDPspeeder's lib/rs.h + lib/fec.h.
 *
 * librsmi.so exports these with C++ linkage and exactly the reference's
 * parameter types, so the mangled symbols match the ones fec_manager.cpp and
 * misc.cpp link against (_Z10rs_encode2iiPPci, _Z10rs_decode2iiPPci, ...).
 * Semantics are the reference's, including decode's in-place pointer
 * permutation (lib/rs.h:25-38); the byte arithmetic runs on the GPU through
 * the batched engine (rsmi.h).  There is no CPU fallback: if no GPU is
 * usable, encode leaves parity untouched and decode returns 1, with a
 * message on stderr.
 *
 *   declaration                                   replaces
 *   void  rs_encode2(int,int,char*[],int)         lib/rs.h:41   (lib/rs.cpp:56-59)
 *   int   rs_decode2(int,int,char*[],int)         lib/rs.h:43   (lib/rs.cpp:61-64)
 *   void  rs_encode(void*,char*[],int)            lib/rs.h:23   (lib/rs.cpp:11-19)
 *   int   rs_decode(void*,char*[],int)            lib/rs.h:39   (lib/rs.cpp:21-40)
 *   void* get_code(int,int)                       lib/rs.cpp:43 (not in rs.h)
 *   void* fec_new(int,int)                        lib/fec.h:47  (lib/fec.cpp:665-720)
 *   void  fec_free(void*)                         lib/fec.h:46  (lib/fec.cpp:648-659)
 *   void  fec_encode(void*,void*[],void*,int,int) lib/fec.h:50  (lib/fec.cpp:727-750)
 *   int   fec_decode(void*,void*[],int[],int)     lib/fec.h:51  (lib/fec.cpp:838-882)
 *   int   get_k(void*) / get_n(void*)             lib/fec.h:53-54 (lib/fec.cpp:883-892)
 */
#ifndef RS_COMPAT_H_
#define RS_COMPAT_H_

#ifndef __cplusplus
#error "rs_compat.h is the C++-linkage drop-in; C callers use rsmi.h"
#endif

void fec_free(void *p);
void *fec_new(int k, int n);
void fec_encode(void *code, void *src[], void *dst, int index, int sz);
int fec_decode(void *code, void *pkt[], int index[], int sz);
int get_k(void *code);
int get_n(void *code);

void rs_encode(void *code, char *data[], int size);
int rs_decode(void *code, char *data[], int size);
void *get_code(int k, int n);
void rs_encode2(int k, int n, char *data[], int size);
int rs_decode2(int k, int n, char *data[], int size);

#endif /* RS_COMPAT_H_ */

/* rocjpeg_version.h -- API version of the drop-in.  Same macro names as the reference's
 * api/rocjpeg_version.h:36-53; the API level implemented is the reference's 0.6.0. */
#ifndef ROCJPEG_VERSION_H
#define ROCJPEG_VERSION_H

#define ROCJPEG_MAJOR_VERSION 0
#define ROCJPEG_MINOR_VERSION 6
#define ROCJPEG_MICRO_VERSION 0

/* true when the library version is >= major.minor.micro (api/rocjpeg_version.h:49-53) */
#define ROCJPEG_CHECK_VERSION(major, minor, micro)                                          \
  (ROCJPEG_MAJOR_VERSION > (major) ||                                                       \
   (ROCJPEG_MAJOR_VERSION == (major) && ROCJPEG_MINOR_VERSION > (minor)) ||                 \
   (ROCJPEG_MAJOR_VERSION == (major) && ROCJPEG_MINOR_VERSION == (minor) &&                 \
    ROCJPEG_MICRO_VERSION >= (micro)))

#endif /* ROCJPEG_VERSION_H */
